// subpixel_wide.hip -- the subpixel refine for stacks of 41-65 images (MAXN 48/56/65: one
// wave per SIMD, register arrays past 256 VGPRs), built with the default SLP vectorisation:
// there the packed f32 schedule measured faster (n = 65: 1.90 vs 2.07 ms scalar).
#include "subpixel.hpp"

namespace bicos_hip {

namespace {

template <typename TIn, typename TPrec>
hipError_t launch_wide_t(const AgreeArgs& a, hipStream_t st) {
    const int n = a.n;
    if (n <= 48) return launch_subpixel_m<TIn, TPrec, 48, 41>(a, st);
    if (n <= 56) return launch_subpixel_m<TIn, TPrec, 56, 49>(a, st);
    if (n <= 65) return launch_subpixel_m<TIn, TPrec, 65, 57>(a, st);
    return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_subpixel_wide(const AgreeArgs& a, int depth, bool dbl, hipStream_t st) {
    if (depth == 1) return dbl ? launch_wide_t<uint8_t, double>(a, st) : launch_wide_t<uint8_t, float>(a, st);
    return dbl ? launch_wide_t<uint16_t, double>(a, st) : launch_wide_t<uint16_t, float>(a, st);
}

}  // namespace bicos_hip
