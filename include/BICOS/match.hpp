// BICOS/match.hpp -- drop-in for the reference's installed <BICOS/match.hpp> (reference
// include/match.hpp:31-41): BICOS::match(stack0, stack1, disparity, cfg = {}, corrmap =
// nullptr) on BICOS::Image, i.e.
//   * with OpenCV: the reference's CPU-build signature on cv::Mat (header-only front end,
//     <bicos/opencv.hpp>: every cv::Mat becomes a zero-copy HipImage view, the outputs are
//     created as S16 / F32 disparity and F32 / F64 corrmap like src/impl/cpu.cpp:77-95),
//   * without OpenCV: the native BICOS::match on HipImage (<bicos/match.hpp>), whose extra
//     trailing hipStream_t defaults to the null stream.
// Either way the gfx950 engine in libbicos_amd.so does the work (link -lbicos_amd, or
// find_package(BICOS) and target_link_libraries(... BICOS::BICOS)).
#pragma once

#include <vector>

#include "common.hpp"

#if defined(BICOS_IMAGE_IS_CV_MAT)
#include "../bicos/opencv.hpp"
#else
#include "../bicos/match.hpp"
#endif
