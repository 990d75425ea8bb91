// BICOS/common.hpp -- drop-in for the reference's installed <BICOS/common.hpp> (reference
// include/common.hpp, installed by CMakeLists.txt:99-104): INVALID_DISP / is_invalid
// (:34-48), Image (:50-56), TransformMode / Precision / Variant / Config (:58-82) and
// Exception (:84-90), all from <bicos/types.hpp>.
//
// `BICOS::Image` is cv::Mat when <opencv2/core.hpp> is available -- exactly the reference's
// CPU build (common.hpp:50-51), so `BICOS::Image disp;` and std::vector<cv::Mat> stacks
// compile unchanged -- and BICOS::HipImage (host or device memory) otherwise. Define
// BICOS_NO_OPENCV to force HipImage. Precision is declared in every build (the reference
// declares it in the CUDA build only); Config::precision defaults to SINGLE.
#pragma once

#include "config.hpp"
#include "../bicos/types.hpp"

#if !defined(BICOS_NO_OPENCV) && defined(__has_include)
#if __has_include(<opencv2/core.hpp>)
#include <opencv2/core.hpp>
#define BICOS_IMAGE_IS_CV_MAT 1
#endif
#endif

namespace BICOS {
#if defined(BICOS_IMAGE_IS_CV_MAT)
using Image = cv::Mat;
#else
using Image = HipImage;
#endif
}  // namespace BICOS
