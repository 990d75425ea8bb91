// subpixel.hip -- the subpixel refine for stacks of up to 40 images, and the dispatch by
// stack depth (launch_subpixel). Built with -fno-slp-vectorize (Makefile): the kernel is
// VALU-issue-bound, and the packed f32 ops the SLP vectoriser forms (v_pk_mul/add/fma_f32)
// issue in two cycles for their two values while their operand pairs cost extra v_mov;
// scalar fp32 is 6-17 % faster for n <= 33. Deeper stacks (one wave per
// SIMD, arrays past 256 registers) run the SLP build: subpixel_wide.hip.
#include "subpixel.hpp"

namespace bicos_hip {

namespace {

// n = 25..33 runs the LDS-staged kernel (subpixel.hpp, NCS) at 3 waves/SIMD instead of the
// register-only one at 2 (213 VGPRs): 0.638 vs 0.676 ms at n = 33 (A/B in one session).
// BICOS_SP33_NCS = the C slots held in LDS with every D0 slot: the fewest that fit 168 VGPRs
// without spills (16: 128 B/lane of scratch); 18 slots + 33 = 51 KiB per 256-thread
// workgroup, 3 per CU. The same staging for n = 17..24 at 4 waves/SIMD (12 C slots, 36 KiB)
// measured 2 % slower than its register-only kernel at 3 waves (0.449 vs 0.441 ms): not used.
#ifndef BICOS_SP33_NCS
#define BICOS_SP33_NCS 18
#endif
template <typename TIn, typename TPrec>
hipError_t launch_subpixel_t(const AgreeArgs& a, int depth, bool dbl, hipStream_t st) {
    const int n = a.n;
    // exact kernels for stack depths the buckets below would pad by a quarter or more: the
    // reference's integration bench (FULL n = 6 / 12, bench/cuda.cu:397-401) and kernel
    // bench (n = 10, bench/cuda.cu:44)
    if (n == 6) return launch_subpixel_m<TIn, TPrec, 6, 6>(a, st);
    if (n == 10) return launch_subpixel_m<TIn, TPrec, 10, 10>(a, st);
    if (n == 12) return launch_subpixel_m<TIn, TPrec, 12, 12>(a, st);
    if (n <= 8) return launch_subpixel_m<TIn, TPrec, 8, 2>(a, st);
    if (n <= 16) return launch_subpixel_m<TIn, TPrec, 16, 9>(a, st);
    if (n <= 24) return launch_subpixel_m<TIn, TPrec, 24, 17>(a, st);
    if (n <= 33) {
        // single precision: the LDS-staged kernel; double keeps every array in registers
        if constexpr (sizeof(TPrec) == 4) return launch_subpixel_m<TIn, TPrec, 33, 25, BICOS_SP33_NCS, 3>(a, st);
        else return launch_subpixel_m<TIn, TPrec, 33, 25>(a, st);
    }
    if (n <= 40) return launch_subpixel_m<TIn, TPrec, 40, 34>(a, st);
    return launch_subpixel_wide(a, depth, dbl, st);
}

}  // namespace

hipError_t launch_subpixel(const AgreeArgs& a, int depth, bool dbl, hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    if (a.nsteps < 1) return hipErrorInvalidValue;
    if (a.fwd) return hipErrorInvalidValue;  // (the Consistency check runs in the agree only)
    if (depth == 1)
        return dbl ? launch_subpixel_t<uint8_t, double>(a, depth, dbl, st)
                   : launch_subpixel_t<uint8_t, float>(a, depth, dbl, st);
    return dbl ? launch_subpixel_t<uint16_t, double>(a, depth, dbl, st)
               : launch_subpixel_t<uint16_t, float>(a, depth, dbl, st);
}

}  // namespace bicos_hip
