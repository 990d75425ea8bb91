// bicos/common.hpp -- the native API's types: everything in bicos/types.hpp, and
// `BICOS::Image` = BICOS::HipImage (host or device memory). Reference callers that include
// the reference's header names instead use include/BICOS/common.hpp, where Image is cv::Mat
// when OpenCV is available; do not include both spellings in one translation unit.
#pragma once

#include "types.hpp"

namespace BICOS {
using Image = HipImage;
}  // namespace BICOS
