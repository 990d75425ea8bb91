// bicos/hip.hpp -- the gfx950 backend behind BICOS::match, at the seam where the reference
// plugs its CPU and CUDA implementations (reference include/cpu.hpp:27-33
// `BICOS::impl::cpu::match`, include/cuda.hpp:27-34 `BICOS::impl::cuda::match`, selected in
// src/lib.cpp:42-48). BICOS::match (bicos/match.hpp) forwards here unconditionally; code
// that called impl::cpu::match / impl::cuda::match directly calls impl::hip::match with the
// same arguments (Image for cv::Mat / cv::cuda::GpuMat, hipStream_t for cv::cuda::Stream).
#pragma once


#include <vector>

#include "types.hpp"

namespace BICOS::impl::hip {

// stack0 / stack1: n single-channel U8 or U16 images of one size, all in host memory or all
// in device memory. Host images: banded pinned upload, match, maps written to host buffers
// (synchronous). Device images: zero-copy when each stack is one planar buffer (equal
// pitches, planes equally spaced), else staged with 2-D copies; the match is enqueued on
// `stream` and the maps are device images (asynchronous).
void match(const std::vector<HipImage>& stack0, const std::vector<HipImage>& stack1, HipImage& disparity,
           Config cfg, HipImage* corrmap, hipStream_t stream);

}  // namespace BICOS::impl::hip
