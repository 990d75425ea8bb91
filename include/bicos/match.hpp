// bicos/match.hpp -- BICOS::match, the drop-in for the reference's public entry
// point (reference include/match.hpp:31-41, src/lib.cpp:31-49).
//
// Backend: always the gfx950 HIP engine (there is no compile-time CPU/CUDA switch
// and no CPU fallback). Inputs may live in host memory (the reference's CPU build,
// Image = cv::Mat) or in device memory (the reference's CUDA build, Image =
// cv::cuda::GpuMat); outputs are allocated in the same memory as the inputs.
//
// Output typing follows the reference CPU path (src/impl/cpu.cpp:77-95):
//   no nxcorr_threshold      -> disparity int16 (S16), invalid = -32768, corrmap untouched
//   nxcorr, no subpixel      -> disparity float32 (F32), invalid = -32768.0f
//   nxcorr + subpixel_step   -> disparity float32, invalid = NaN
//   corrmap (when requested and nxcorr set): float32, NaN where not evaluated
//   (float64 with Precision::DOUBLE, as the reference CUDA build, cuda.cu:217)
//
// Errors throw BICOS::Exception (including "input stacks too large", which the
// reference raised as std::invalid_argument, cpu.cpp:155).
#pragma once


#include <vector>

#include "types.hpp"

namespace BICOS {

void match(const std::vector<HipImage>& stack0, const std::vector<HipImage>& stack1, HipImage& disparity,
           Config cfg = Config{}, HipImage* corrmap = nullptr, hipStream_t stream = nullptr);

}  // namespace BICOS
