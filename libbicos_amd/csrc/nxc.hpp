// nxc.hpp -- device helpers of the NXC agree (reference include/impl/cpu/agree.hpp:28-93)
// shared by the agree kernels (kernels.hip) and the subpixel refine (subpixel.hpp).
//
// Numerics: every float op is an explicit IEEE round-to-nearest op (the sources are compiled
// with -ffp-contract=off), fmaf exactly where the reference calls std::fmaf, correctly
// rounded division and sqrt.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bicos_hip {
namespace nxc {

template <typename T>
__device__ __forceinline__ uint32_t ld(const T* p) {
    return (uint32_t)__builtin_nontemporal_load(p);
}

__device__ __forceinline__ float fma_p(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_p(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float div_p(float a, float b) { return __fdiv_rn(a, b); }
__device__ __forceinline__ double div_p(double a, double b) { return __ddiv_rn(a, b); }
// Correctly rounded sqrtf. hipcc lowers __fsqrt_rn / sqrtf to a bare v_sqrt_f32 (up to
// 1 ulp off) here; the reference's std::sqrt is IEEE. Fix the estimate s with the residuals
// of its two float neighbours (x - s_dn*s <= 0 -> s_dn; x - s_up*s > 0 -> s_up), after
// scaling tiny inputs into the normal range.
__device__ __forceinline__ float sqrt_p(float x) {
    const bool tiny = x < 0x1.0p-96f;
    const float xs = tiny ? x * 0x1.0p+32f : x;
    float s = __builtin_amdgcn_sqrtf(xs);
    const int si = __float_as_int(s);
    const float s_dn = __int_as_float(si - 1);
    const float s_up = __int_as_float(si + 1);
    const float r_dn = __builtin_fmaf(-s_dn, s, xs);
    const float r_up = __builtin_fmaf(-s_up, s, xs);
    s = r_dn <= 0.f ? s_dn : s;
    s = r_up > 0.f ? s_up : s;
    s = tiny ? s * 0x1.0p-16f : s;
    // zero, +inf and NaN (and negative) pass through the hardware result
    return (xs == 0.f || xs == __builtin_inff() || !(xs > 0.f)) ? __builtin_amdgcn_sqrtf(x) : s;
}
__device__ __forceinline__ double sqrt_p(double a) { return __dsqrt_rn(a); }
// sqrt_p for x = 0 or 2^-96 <= x < +inf only -- the product of two variances of integer
// samples (each 0 or >= (1/65)^2, see subpixel.hpp) -- without the tiny-input scaling and the
// special-value select: x = 0 gives s = 0 (r_dn is NaN, r_up is 0: neither fix-up fires)
__device__ __forceinline__ float sqrt_p_var(float x) {
    float s = __builtin_amdgcn_sqrtf(x);
    const int si = __float_as_int(s);
    const float s_dn = __int_as_float(si - 1);
    const float s_up = __int_as_float(si + 1);
    const float r_dn = __builtin_fmaf(-s_dn, s, x);
    const float r_up = __builtin_fmaf(-s_up, s, x);
    s = r_dn <= 0.f ? s_dn : s;
    return r_up > 0.f ? s_up : s;
}
__device__ __forceinline__ double sqrt_p_var(double a) { return __dsqrt_rn(a); }

// s / n correctly rounded for an integer-valued s in [0, 65535 n] and 2 <= n <= 65, given
// rn = RN(1 / n): q0 = RN(s rn), r = s - q0 n (exact by fma), RN(q0 + r rn). Checked
// against IEEE division for every such (s, n) -- 1.4e8 cases, no difference
// (tools/div_by_n_check.c). Three full-rate ops instead of the ~10 of a correctly rounded
// division; the means of u8 / u16 samples (sums < 2^24) are exactly these quotients.
__device__ __forceinline__ float div_by_n(float s, float nf, float rn) {
    const float q0 = s * rn;
    const float r = __builtin_fmaf(-q0, nf, s);
    return __builtin_fmaf(r, rn, q0);
}

// nxcorr (agree.hpp:28-51): means from exact integer sums (< 2^24, identical to the
// reference's sequential float sums); centred samples, three fma chains in t order,
// IEEE sqrt and division. TPrec = double is the CUDA build's Precision::DOUBLE
// (agree.cuh:35-65), which has no CPU counterpart in the reference.
template <typename TIn, typename TPrec>
__device__ __forceinline__ TPrec nxcorr_dev(const TIn* __restrict__ p0, const TIn* __restrict__ p1,
                                           size_t pp, int n, bool has_minvar, TPrec minvar) {
    uint32_t s0 = 0, s1 = 0;
    for (int t = 0; t < n; ++t) {
        s0 += ld(p0 + t * pp);
        s1 += ld(p1 + t * pp);
    }
    const TPrec m0 = div_p((TPrec)s0, (TPrec)n);
    const TPrec m1 = div_p((TPrec)s1, (TPrec)n);
    TPrec cov = 0, v0 = 0, v1 = 0;
    for (int t = 0; t < n; ++t) {
        const TPrec x0 = (TPrec)ld(p0 + t * pp) - m0;
        const TPrec x1 = (TPrec)ld(p1 + t * pp) - m1;
        cov = fma_p(x0, x1, cov);
        v0 = fma_p(x0, x0, v0);
        v1 = fma_p(x1, x1, v1);
    }
    if (has_minvar && (v0 < minvar || v1 < minvar)) return (TPrec)-1;
    return div_p(cov, sqrt_p(v0 * v1));
}

// The agree of R pixels of one row at once (agree.hpp:53-93 with nxcorr agree.hpp:28-51 in
// single precision): pixel r is column c0[r] of the left row, matched to column best[r] of
// the right row; `in[r]` = the pixel exists, `live[r]` = its search result is valid (then
// best[r] is inside the row, so the NXC always runs). Writes the float disparity
// (c0 - best, -32768 when invalid or below the threshold; NaN correlations pass) and, if
// `corr`, the correlation (NaN for invalid pixels, -1 below the minimum variance).
// The R pixels go through each of the two passes together, so each pass is one round of
// loads in flight instead of R. `minvar` is already scaled by n (cpu.cpp:127).
template <typename TIn, int R>
__device__ __forceinline__ void agree_pixels(const TIn* s0, const TIn* s1, size_t pp, int n,
                                             const int (&c0)[R], const int (&best)[R],
                                             const bool (&in)[R], const bool (&live)[R],
                                             float threshold, bool has_minvar, float minvar,
                                             float* outf, float* corr) {
    const TIn* p0[R];
    const TIn* p1[R];
    uint32_t sl[R], sr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        p0[r] = s0 + (in[r] ? c0[r] : 0);
        p1[r] = s1 + (live[r] ? best[r] : 0);
        sl[r] = 0;
        sr[r] = 0;
    }
    for (int t = 0; t < n; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            sl[r] += ld(p0[r] + t * pp);
            sr[r] += ld(p1[r] + t * pp);
        }
    float m0[R], m1[R], cov[R], v0[R], v1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        m0[r] = div_p((float)sl[r], (float)n);
        m1[r] = div_p((float)sr[r], (float)n);
        cov[r] = v0[r] = v1[r] = 0.f;
    }
    for (int t = 0; t < n; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float x0 = (float)ld(p0[r] + t * pp) - m0[r];
            const float x1 = (float)ld(p1[r] + t * pp) - m1[r];
            cov[r] = fma_p(x0, x1, cov[r]);
            v0[r] = fma_p(x0, x0, v0[r]);
            v1[r] = fma_p(x1, x1, v1[r]);
        }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!in[r]) continue;
        float o = -32768.f;
        float cr = __builtin_nanf("");
        if (live[r]) {
            if (has_minvar && (v0[r] < minvar || v1[r] < minvar))
                cr = -1.f;
            else
                cr = div_p(cov[r], sqrt_p(v0[r] * v1[r]));
            if (!(cr < threshold)) o = (float)(c0[r] - best[r]);  // NaN passes
        }
        outf[c0[r]] = o;
        if (corr) corr[c0[r]] = cr;
    }
}

}  // namespace nxc
}  // namespace bicos_hip
