// subpixel.hpp -- agree_subpixel (reference include/impl/cpu/agree.hpp:95-191): NXC of the
// integer match plus the quadratic refine over x = -1, -1 + step, ... <= 1. The kernel
// template is instantiated in two translation units: subpixel.hip (MAXN <= 40, built
// without SLP vectorisation: scalar fp32 only) and subpixel_wide.hip (MAXN >= 48, built
// with it), see the Makefile.
#pragma once

#include "kernels.hpp"
#include "nxc.hpp"
#include "stack.hpp"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bicos_hip {
namespace {

constexpr int16_t SP_INVALID_I16 = -32768;
using nxc::div_p;
using nxc::fma_p;
using nxc::nxcorr_dev;
using nxc::sqrt_p;

// (TIn)roundevenf(A x^2 + B x + C) as a float (agree.cuh:221-236 / agree.hpp:140-150):
// adding 1.5*2^23 rounds v to the nearest even integer k (|v| < 2^22 for 8/16-bit data)
// and leaves k's two's-complement low bits in the mantissa, so the low byte/short of the
// sum's bits IS (TIn)(int)k, the reference's wrap through int32. It goes back to float
// exactly as (2^23 | low bits) - 2^23; the sum's top byte is always 0x4B, so that is one
// full-rate AND with 0x4B0000FF (0x4B00FFFF) and a subtract, instead of the quarter-rate
// v_cvt_f32_ubyte0 (tools/valu_peak.hip, op 19).
constexpr float RND_MAGIC = 0x1.8p23f;

// (float)k for |k| < 2^22, exactly: full-rate integer add + float subtract
__device__ __forceinline__ float small_int_to_float(int k) {
    uint32_t b = 0x4B400000u + (uint32_t)k;
    asm("" : "+v"(b));  // keep LLVM from folding this back into v_cvt_f32_i32
    return __uint_as_float(b) - RND_MAGIC;
}
template <typename TIn>
constexpr uint32_t wrap_mask() { return sizeof(TIn) == 1 ? 0x4B0000FFu : 0x4B00FFFFu; }

template <typename TIn>
__device__ __forceinline__ float interp_wrapped(float A, float B, float C, float x) {
    const float ax = A * x;
    const float v = (ax * x + B * x) + C;
    uint32_t bits = __float_as_uint(v + RND_MAGIC) & wrap_mask<TIn>();
    asm("" : "+v"(bits));  // keep LLVM from folding this back into a cvt
    return __uint_as_float(bits) - 0x1p23f;
}

// agree_subpixel (agree.hpp:95-191). MAXN >= n bounds the per-lane register arrays
// (static indices only). Slots t < LO (the smallest n routed to this bucket) are always
// live; slots LO <= t < MAXN beyond n are padded with exact no-ops: A = B = C = 0 gives
// an interpolated 0 (sum unchanged), D0 = 0 and x1 = 0 leave both fma chains unchanged
// (neither accumulator is ever -0). The quadratic is float in both precisions.
//
// The x loop is software-pipelined: one pass over t finishes step k (x1 = IV - m1 and the
// in-order cov / var fma chains) and interpolates step k+1 into the same IV registers, so
// every chain op has independent interpolation work beside it and the register footprint
// is that of one step. nsteps is the host's count of x = -1, -1+step, ... <= 1, accumulated
// in float exactly as the reference's loop (engine.cpp subpixel_steps).
// NCS >= 0 (float, MAXN <= 40): the centred left samples D0 of every slot and the C of the
// top NCS slots live in LDS instead of registers ([slot][thread], one conflict-free
// ds_read_b32 with an immediate offset per use; each thread reads only what it wrote, so no
// barrier), which brings the kernel under WPE waves/SIMD's register budget. The arithmetic
// is unchanged.
template <typename TIn, typename TPrec, int MAXN, int LO, int NCS = -1, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void subpixel_kernel(AgreeArgs a) {
    constexpr bool STG = NCS >= 0;
    static_assert(!STG || (sizeof(TPrec) == 4 && MAXN <= 40 && NCS <= MAXN), "LDS staging: float, n <= 40");
    constexpr int CS = MAXN - (NCS > 0 ? NCS : 0);  // first C slot held in LDS
    __shared__ float sD0[STG ? MAXN : 1][256];
    __shared__ float sC[STG && NCS > 0 ? NCS : 1][256];
    const int tid = threadIdx.x;
    int tile, row;
    xcd_rows(tile, row);
    const int col = tile * 256 + threadIdx.x;
    if (col >= a.cols) return;
    const size_t o = (size_t)row * a.cols + col;
    const int n = LO == MAXN ? MAXN : a.n;
    const size_t pp = a.plane_pitch;
    const int d = a.raw[(size_t)row * a.raw_pitch + col];
    const TPrec minvar = (TPrec)a.minvar;
    float out = __builtin_nanf("");
    TPrec corr = (TPrec)__builtin_nan("");
    const int col1 = col - d;
    if (d != SP_INVALID_I16 && col1 >= 0 && col1 < a.cols) {
        const TIn* s0 = (const TIn*)a.stack0 + (size_t)row * a.row_pitch + col;
        const TIn* s1 = (const TIn*)a.stack1 + (size_t)row * a.row_pitch + col1;
        if (col1 == 0 || col1 == a.cols - 1) {
            corr = nxcorr_dev<TIn, TPrec>(s0, s1, pp, n, a.has_minvar, minvar);
            if (!(corr < (TPrec)a.threshold)) out = (float)d;
        } else {
            const StackReader<TIn> rd0(a.stack0, a.stack_bytes), rd1(a.stack1, a.stack_bytes);
            const uint32_t rowoff = (uint32_t)row * (uint32_t)a.row_pitch;
            // left: mean, centred samples and variance are the same for every x
            // padded slots re-read plane 0 (in bounds) and are zeroed; int -> float via
            // small_int_to_float (two full-rate ops instead of a quarter-rate v_cvt_f32_*)
            TPrec D0[STG ? 1 : MAXN];
            float A[MAXN], B[MAXN], C[MAXN];
            uint32_t s = 0;
#pragma unroll
            for (int t = 0; t < MAXN; ++t) {
                const bool live = t < LO || t < n;
                const uint32_t po = rowoff + (live ? (uint32_t)(t * pp) : 0u);
                const uint32_t l = rd0((uint32_t)col, po);
                const int y0 = (int)rd1((uint32_t)(col1 - 1), po);
                const int y1 = (int)rd1((uint32_t)col1, po);
                const int y2 = (int)rd1((uint32_t)(col1 + 1), po);
                // 0.5f * ( y0 - 2.0f * y1 + y2) ; 0.5f * (-y0 + y2) ; y1 -- exact on integers
                // of this size, so formed in int and converted once
                A[t] = live ? 0.5f * small_int_to_float(y0 - 2 * y1 + y2) : 0.f;
                B[t] = live ? 0.5f * small_int_to_float(y2 - y0) : 0.f;
                C[t] = live ? small_int_to_float(y1) : 0.f;
                const TPrec lf = live ? (TPrec)small_int_to_float((int)l) : (TPrec)0;
                if constexpr (STG) {
                    sD0[t][tid] = lf;  // the raw sample; centred below
                    if (t >= CS) sC[t >= CS ? t - CS : 0][tid] = C[t];
                    // at most 8 slots' loads in flight: the prologue stays inside the
                    // 168-register budget of 3 waves/SIMD too
                    if (t % 8 == 7) asm volatile("" ::: "memory");
                } else {
                    D0[t] = lf;
                }
                s += live ? l : 0u;
            }
            // The empty asm statements with a memory clobber (here, and at the top of every x
            // step) stop the compiler from forwarding stored values or hoisting the
            // loop-invariant LDS reads, either of which would keep the arrays in registers.
            if constexpr (STG) asm volatile("" ::: "memory");
            const TPrec m0 = div_p((TPrec)s, (TPrec)n);
            const float rn = div_p(1.f, (float)n);  // RN(1/n) for nxc::div_by_n
            TPrec v0 = 0;
#pragma unroll
            for (int t = 0; t < MAXN; ++t) {
                const bool live = t < LO || t < n;
                if constexpr (STG) {
                    const TPrec dc = live ? sD0[t][tid] - m0 : (TPrec)0;
                    sD0[t][tid] = dc;
                    v0 = fma_p(dc, dc, v0);
                } else {
                    D0[t] = live ? D0[t] - m0 : (TPrec)0;
                    v0 = fma_p(D0[t], D0[t], v0);
                }
            }
            if constexpr (STG) asm volatile("" ::: "memory");
            const bool v0_low = a.has_minvar && v0 < minvar;
            // the left sample / C of slot t: registers, or this thread's LDS slot
            auto d0_of = [&](int t) -> TPrec {
                if constexpr (STG) return sD0[t][tid];
                else return D0[t];
            };
            auto c_of = [&](int t) -> float {
                if constexpr (STG) {
                    if (t >= CS) return sC[t >= CS ? t - CS : 0][tid];
                }
                return C[t];
            };

            float best_x = 0.f;
            TPrec best = -1;
            const float step = a.step;
            float x = -1.f;
            // cov / var of step x, then the reference's argmax (first maximum wins)
            auto finish = [&](TPrec cov, TPrec v1) {
                TPrec nxc;
                if (v0_low || (a.has_minvar && v1 < minvar))
                    nxc = -1;
                else
                    // v0, v1: 0 or >= (1/65)^2 (centred integer samples: |l - m| is 0 or
                    // >= ~1/n), so their product is 0 or far above 2^-96
                    nxc = div_p(cov, nxc::sqrt_p_var(v0 * v1));
                if (best < nxc) {
                    best_x = x;
                    best = nxc;
                }
            };
            float IV[MAXN];
            float sf[4] = {0.f, 0.f, 0.f, 0.f};  // exact in any order: integers < 2^24
            if constexpr (MAXN <= 40) {
                // Software-pipelined: one pass over t finishes step k (x1 = IV - m1 and the
                // in-order fma chains) and interpolates step k+1 into the same registers.
#pragma unroll
                for (int t = 0; t < MAXN; ++t) {
                    IV[t] = interp_wrapped<TIn>(A[t], B[t], c_of(t), x);
                    sf[t & 3] += IV[t];
                }
                for (int k = 0; k < a.nsteps; ++k) {
                    if constexpr (STG) asm volatile("" ::: "memory");
                    const float sum = (sf[0] + sf[1]) + (sf[2] + sf[3]);
                    TPrec m1;
                    if constexpr (sizeof(TPrec) == 4)
                        m1 = nxc::div_by_n(sum, (float)n, rn);
                    else
                        m1 = div_p((TPrec)sum, (TPrec)n);
                    const float xn = x + step;
                    TPrec cov = 0, v1 = 0;
                    // two copies of the body: a wave-uniform test inside the unrolled t loop
                    // becomes one scalar branch per slot and breaks the schedule (measured 3x)
                    if (k + 1 < a.nsteps) {
#pragma unroll
                        for (int t = 0; t < MAXN; ++t) {
                            TPrec x1 = (TPrec)IV[t] - m1;
                            if (t >= LO) x1 = t < n ? x1 : (TPrec)0;
                            cov = fma_p(d0_of(t), x1, cov);
                            v1 = fma_p(x1, x1, v1);
                            IV[t] = interp_wrapped<TIn>(A[t], B[t], c_of(t), xn);
                        }
                        sf[0] = sf[1] = sf[2] = sf[3] = 0.f;
#pragma unroll
                        for (int t = 0; t < MAXN; ++t) sf[t & 3] += IV[t];
                    } else {
#pragma unroll
                        for (int t = 0; t < MAXN; ++t) {
                            TPrec x1 = (TPrec)IV[t] - m1;
                            if (t >= LO) x1 = t < n ? x1 : (TPrec)0;
                            cov = fma_p(d0_of(t), x1, cov);
                            v1 = fma_p(x1, x1, v1);
                        }
                    }
                    finish(cov, v1);
                    x = xn;
                }
            } else {
                // One wave/SIMD: the arrays already overflow into AGPRs, so keep IV dead
                // across the loop's back edge (interpolate at the top of each step).
                for (int k = 0; k < a.nsteps; ++k) {
                    sf[0] = sf[1] = sf[2] = sf[3] = 0.f;
#pragma unroll
                    for (int t = 0; t < MAXN; ++t) {
                        IV[t] = interp_wrapped<TIn>(A[t], B[t], C[t], x);
                        sf[t & 3] += IV[t];
                    }
                    const TPrec m1 = div_p((TPrec)((sf[0] + sf[1]) + (sf[2] + sf[3])), (TPrec)n);
                    TPrec cov = 0, v1 = 0;
#pragma unroll
                    for (int t = 0; t < MAXN; ++t) {
                        TPrec x1 = (TPrec)IV[t] - m1;
                        if (t >= LO) x1 = t < n ? x1 : (TPrec)0;
                        cov = fma_p(D0[t], x1, cov);
                        v1 = fma_p(x1, x1, v1);
                    }
                    finish(cov, v1);
                    x += step;
                }
            }
            corr = best;
            if (!(best < (TPrec)a.threshold)) out = (float)d - best_x;
        }
    }
    ((float*)a.out)[o] = out;
    if (a.corrmap) ((TPrec*)a.corrmap)[o] = corr;
}

template <typename TIn, typename TPrec, int MAXN, int LO, int NCS = -1, int WPE = 1>
hipError_t launch_subpixel_m(const AgreeArgs& a, hipStream_t st) {
    dim3 grid((a.cols + 255) / 256, a.rows);
    if (a.n == MAXN)
        hipLaunchKernelGGL((subpixel_kernel<TIn, TPrec, MAXN, MAXN, NCS, WPE>), grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((subpixel_kernel<TIn, TPrec, MAXN, LO, NCS, WPE>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace
}  // namespace bicos_hip
