// bicos/opencv.hpp -- header-only OpenCV front end: the reference's signature
// BICOS::match(const std::vector<cv::Mat>&, const std::vector<cv::Mat>&, cv::Mat&, Config,
// cv::Mat*) (reference include/match.hpp:31-41, CPU build) on top of the gfx950 engine, so
// reference C++ callers compile unchanged when OpenCV is installed.
//
// The conversion is a template over any host matrix type with OpenCV's members (rows, cols,
// data, step[0], type(), create(rows, cols, type)) -- `match_mats` -- and the cv::Mat
// overload below is that template instantiated for cv::Mat, compiled only when
// <opencv2/core.hpp> is available. No pixel is copied on the way in: every cv::Mat becomes
// a BICOS::Image view; the outputs are created through the caller's matrix type (S16 or F32
// disparity, F32 / F64 corrmap, reference src/impl/cpu.cpp:77-95) and written in place.
#pragma once

#include <vector>

#include "hip.hpp"
#include "types.hpp"

namespace BICOS {

template <class MatT>
HipImage image_view(const MatT& m) {
    return HipImage(m.rows, m.cols, m.type(), (void*)m.data, (size_t)m.step[0], Memory::Host);
}

template <class MatT>
void match_mats(const std::vector<MatT>& stack0, const std::vector<MatT>& stack1,
                MatT& disparity, Config cfg = Config{}, MatT* corrmap = nullptr) {
    std::vector<HipImage> s0, s1;
    s0.reserve(stack0.size());
    s1.reserve(stack1.size());
    for (const MatT& m : stack0) s0.push_back(image_view(m));
    for (const MatT& m : stack1) s1.push_back(image_view(m));
    if (stack0.empty() || stack1.empty()) {
        HipImage d;
        impl::hip::match(s0, s1, d, cfg, nullptr, nullptr);  // throws the reference's error
        return;
    }
    const int rows = stack0.front().rows, cols = stack0.front().cols;
    const bool nxc = cfg.nxcorr_threshold.has_value();
    // allocate the outputs in the caller's type first, then let the engine fill them
    disparity.create(rows, cols, nxc ? (int)F32 : (int)S16);
    HipImage d = image_view(disparity);
    HipImage c;
    if (corrmap && nxc) {
        corrmap->create(rows, cols, cfg.precision == Precision::DOUBLE ? (int)F64 : (int)F32);
        c = image_view(*corrmap);
    }
    impl::hip::match(s0, s1, d, cfg, corrmap && nxc ? &c : nullptr, nullptr);
}

}  // namespace BICOS

#if defined(__has_include)
#if __has_include(<opencv2/core.hpp>)
#include <opencv2/core.hpp>

namespace BICOS {

inline void match(const std::vector<cv::Mat>& stack0, const std::vector<cv::Mat>& stack1,
                  cv::Mat& disparity, Config cfg = Config{}, cv::Mat* corrmap = nullptr) {
    match_mats<cv::Mat>(stack0, stack1, disparity, cfg, corrmap);
}

}  // namespace BICOS
#endif
#endif
