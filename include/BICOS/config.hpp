// BICOS/config.hpp -- the reference's generated build configuration (reference
// cmake/config.hpp.in, installed as include/BICOS/config.hpp by CMakeLists.txt:99-104),
// for the gfx950 HIP build of libbicos_amd. The reference defines BICOS_CPU or BICOS_CUDA
// here; this build defines BICOS_HIP and neither of those: its host API is the reference's
// CPU-build signature (cv::Mat in, cv::Mat out, no stream argument) served by the GPU, plus
// the device-resident HipImage / hipStream_t entry points of <bicos/match.hpp>.
#pragma once

#define BICOS_VERSION "2.2.0"
#define BICOS_HIP 1
