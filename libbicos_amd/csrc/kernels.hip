// kernels.hip -- gfx950 (CDNA4) kernels of the BICOS hot path.
//
//   transform_kernel    descriptor_transform  (reference include/impl/cpu/descriptor_transform.hpp:31-138)
//   search_kernel       bicos Hamming search  (reference include/impl/cpu/bicos.hpp:29-113)
//   consistency_kernel  left-right check      (reference include/impl/cpu/bicos.hpp:99-106)
//   agree_kernel        NXC filter            (reference include/impl/cpu/agree.hpp:28-93)
//   subpixel_kernel     NXC + quadratic refine(reference include/impl/cpu/agree.hpp:95-191)
//
// Layouts in HBM (see DESIGN.md "Data layout"):
//   image stack   planar [n][rows][row_pitch] of u8/u16 (the reference's vector<Image>)
//   descriptors   [rows][desc_pitch] uint32, pixel c at words [c*WORDS, c*WORDS+WORDS),
//                 desc_pitch = round_up(cols*WORDS, 4) so every row starts 16-B aligned
//   disparity     int16 [rows][cols] or float32 [rows][cols], dense
//
// Numerics: compiled with -ffp-contract=off; every float op below that the reference
// performs is an explicit IEEE round-to-nearest op (no contraction, correctly rounded
// division and sqrt), fmaf exactly where the reference calls std::fmaf.
#include "kernels.hpp"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bicos_hip {

namespace {

constexpr int16_t INVALID_I16 = -32768;

__device__ __forceinline__ float fdiv_rn(float a, float b) { return __fdiv_rn(a, b); }

// popcount(x) + acc as ONE v_bcnt_u32_b32. Left alone, hipcc re-associates the per-word
// counts into a tree with an extra v_add3 per pair; an instruction-free asm makes the
// accumulator opaque so the chain survives. (A real `v_bcnt` asm statement costs an
// `s_nop` hazard pad per use; this form emits nothing.)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    asm("" : "+v"(acc));
    return __builtin_popcount(x) + acc;
}

// median of three -> v_med3_u32 (pattern-matched by the backend)
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    return max(min(a, b), min(max(a, b), c));
}

template <typename T>
__device__ __forceinline__ uint32_t ld(const T* p) {
    return (uint32_t)__builtin_nontemporal_load(p);
}

// ------------------------------------------------------------------ transform

// Sequential bit writer: bit i of the descriptor is the i-th comparison, LSB first
// (reference include/impl/cpu/bitfield.hpp:34-58). The bit position is wave-uniform,
// so the flush branch is scalar and `w[]` stays in registers (static indices only).
template <int WORDS>
struct BitWriter {
    uint32_t w[WORDS];
    uint32_t cur = 0;
    int nbits = 0;
    int widx = 0;

    __device__ __forceinline__ BitWriter() {
#pragma unroll
        for (int k = 0; k < WORDS; ++k) w[k] = 0;
    }
    __device__ __forceinline__ void flush() {
#pragma unroll
        for (int k = 0; k < WORDS; ++k)
            if (k == widx) w[k] = cur;
    }
    __device__ __forceinline__ void set(bool v) {
        cur |= (uint32_t)v << nbits;
        if (++nbits == 32) {
            flush();
            ++widx;
            cur = 0;
            nbits = 0;
        }
    }
    __device__ __forceinline__ void finish() {
        if (nbits) flush();
    }
};

template <typename TIn, int WORDS, int MODE>
__global__ __launch_bounds__(256) void transform_kernel(TransformArgs a) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y;
    const int which = blockIdx.z;
    if (col >= a.cols) return;
    const TIn* __restrict__ p = (const TIn*)(which ? a.stack1 : a.stack0) + (size_t)row * a.row_pitch + col;
    uint32_t* __restrict__ out = (which ? a.desc1 : a.desc0) + (size_t)row * a.desc_pitch + (size_t)col * WORDS;
    const size_t pp = a.plane_pitch;
    const int n = a.n;

    // Mean: the reference sums as float sequentially then divides (float). The inputs
    // are integers and every partial sum is < 2^24 (n <= 65, values <= 65535), so the
    // float sum is exact and equals the integer sum.
    uint32_t sum = 0;
    for (int t = 0; t < n; ++t) sum += ld(p + t * pp);
    const float av = fdiv_rn((float)sum, (float)n);

    BitWriter<WORDS> bw;
    if (MODE == 0) {
        // LIMITED (descriptor_transform.hpp:31-73). ps(t) = p[t] + p[t+1]; the reference's
        // two-slot ring of previous pair sums equals the shift pair (pm2, pm1) here.
        uint32_t a0 = ld(p), b0 = ld(p + pp);
        int pm1 = -1, pm2 = -1;
        for (int t = 0; t < n - 2; ++t) {
            const uint32_t c0 = ld(p + (t + 2) * pp);
            bw.set(a0 < b0);
            bw.set(a0 < c0);
            bw.set((float)a0 < av);
            const int cur = (int)(a0 + b0);
            if (t >= 2) bw.set(pm2 < cur);
            pm2 = pm1;
            pm1 = cur;
            a0 = b0;
            b0 = c0;
        }
        bw.set(a0 < b0);
        bw.set((float)a0 < av);
        bw.set((float)b0 < av);
        bw.set(pm2 < (int)(a0 + b0));
    } else {
        // FULL (descriptor_transform.hpp:75-123); n <= 16 so the pair sums live in
        // registers with static indices.
        uint32_t ps[15];
#pragma unroll
        for (int t = 0; t < 15; ++t) ps[t] = 0;
        uint32_t a0 = ld(p), b0 = ld(p + pp);
#pragma unroll
        for (int t = 0; t < 14; ++t) {
            if (t < n - 2) {
                const uint32_t c0 = ld(p + (t + 2) * pp);
                bw.set(a0 < b0);
                bw.set(a0 < c0);
                bw.set((float)a0 < av);
                ps[t] = a0 + b0;
                a0 = b0;
                b0 = c0;
            }
        }
#pragma unroll
        for (int t = 0; t < 15; ++t)
            if (t == n - 2) ps[t] = a0 + b0;
        bw.set(a0 < b0);
        bw.set((float)a0 < av);
        bw.set((float)b0 < av);
#pragma unroll
        for (int t = 0; t < 15; ++t)
#pragma unroll
            for (int i = 0; i < 15; ++i)
                if (t < n - 1 && i < n - 1 && i != t && i != t - 1 && i != t + 1)
                    bw.set(ps[t] < ps[i]);
    }
    bw.finish();

    if (WORDS % 4 == 0) {
#pragma unroll
        for (int k = 0; k < WORDS; k += 4)
            *(uint4*)(out + k) = make_uint4(bw.w[k], bw.w[k + 1], bw.w[k + 2], bw.w[k + 3]);
    } else if (WORDS == 2) {
        *(uint2*)out = make_uint2(bw.w[0], bw.w[1 % WORDS]);
    } else {
        out[0] = bw.w[0];
    }
}

// --------------------------------------------------------------------- search

// Hamming cost of one (col0, col1) pair.
template <int WORDS>
__device__ __forceinline__ uint32_t ham(const uint32_t (&a)[WORDS], const uint32_t (&b)[WORDS]) {
    uint32_t c = __builtin_popcount(a[0] ^ b[0]);
#pragma unroll
    for (int k = 1; k < WORDS; ++k) c = bcnt_acc(a[k] ^ b[k], c);
    return c;
}

template <int WORDS>
__device__ __forceinline__ void lds_fetch(const uint32_t* s, uint32_t (&d)[WORDS]) {
    if (WORDS >= 4) {
#pragma unroll
        for (int k = 0; k < WORDS; k += 4) {
            const uint4 v = *(const uint4*)(s + k);
            d[k] = v.x;
            d[(k + 1) % WORDS] = v.y;
            d[(k + 2) % WORDS] = v.z;
            d[(k + 3) % WORDS] = v.w;
        }
    } else if (WORDS == 2) {
        const uint2 v = *(const uint2*)s;
        d[0] = v.x;
        d[1 % WORDS] = v.y;
    } else {
        d[0] = s[0];
    }
}

template <int WORDS, bool NODUPES, int R>
__device__ __forceinline__ void search_step(const uint32_t* s, uint32_t c1,
                                            const uint32_t (&d0)[R][WORDS], uint32_t (&best)[R],
                                            uint32_t (&second)[R]) {
    uint32_t d1[WORDS];
    lds_fetch<WORDS>(s, d1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t key = (ham<WORDS>(d0[r], d1) << 16) | c1;
        if (NODUPES) second[r] = umed3(best[r], key, second[r]);
        best[r] = min(best[r], key);
    }
}

// One workgroup = one (row, col0 tile). The tile's WAVES*64*R left descriptors live in
// registers (R per lane, lanes on consecutive columns); the right row is staged through
// LDS in chunks of `chunk` columns and read back as wave-uniform broadcasts. For every
// col1 each lane updates, per held col0,
//     key    = cost << 16 | col1                     (v_lshl_or_b32, col1 in an SGPR)
//     second = med3(best, key, second)              (v_med3_u32)
//     best   = min(best, key)                       (v_min_u32)
// so `best` is the argmin with the lowest col1 among equal costs (the reference's strict
// '<' scan) and the minimum is duplicated iff cost(second) == cost(best).
//   out_mode 0: out = col0 - best_col1 (INVALID_I16 when rejected)      [disparity]
//   out_mode 1: out = best_col1 (-1 when rejected)                      [Consistency passes]
template <int WORDS, bool NODUPES, int R>
__global__ __launch_bounds__(512) void search_kernel(SearchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    // XCD-aware tile order: hardware deals workgroups round-robin over the 8 XCDs; give
    // each XCD a contiguous range of (row, tile) so the tiles of one row share one L2.
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int per_xcd = (nwg + 7) / 8;
    int logical = (bid % 8) * per_xcd + bid / 8;
    // grids whose size is not a multiple of 8 leave holes at the end of the last XCDs'
    // ranges; fold them back onto the identity map so the mapping stays a bijection
    if (nwg % 8 != 0) logical = bid;
    const int row = logical / a.tiles_per_row;
    const int tile = logical % a.tiles_per_row;

    const int waves = blockDim.x / 64;
    const int wave = threadIdx.x / 64;
    const int lane = threadIdx.x % 64;
    const int cols = a.cols;
    const int col0_base = tile * waves * 64 * R + wave * 64 * R + lane;

    const uint32_t* __restrict__ row0 = a.desc0 + (size_t)row * a.desc_pitch;
    const uint32_t* __restrict__ row1 = a.desc1 + (size_t)row * a.desc_pitch;

    uint32_t d0[R][WORDS];
    uint32_t best[R], second[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int c0 = col0_base + r * 64;
        const int cc = c0 < cols ? c0 : cols - 1;
        lds_fetch<WORDS>(row0 + (size_t)cc * WORDS, d0[r]);
        best[r] = 0xFFFFFFFFu;
        second[r] = 0xFFFFFFFFu;
    }

    for (int base = 0; base < cols; base += a.chunk) {
        const int ncols = min(a.chunk, cols - base);
        const int nwords = ncols * WORDS;
        if (base) __syncthreads();
        {
            const uint32_t* src = row1 + (size_t)base * WORDS;
            const int n4 = nwords / 4;
            for (int i = threadIdx.x; i < n4; i += blockDim.x)
                ((uint4*)lds)[i] = ((const uint4*)src)[i];
            for (int i = n4 * 4 + threadIdx.x; i < nwords; i += blockDim.x) lds[i] = src[i];
        }
        __syncthreads();

        // Static-count inner unroll: the bcnt asm is convergent, which forbids the
        // compiler's runtime unrolling; U LDS broadcasts are issued ahead of the VALU.
        constexpr int U = WORDS >= 8 ? 4 : 8;
        int j = 0;
        for (; j + U <= ncols; j += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) search_step<WORDS, NODUPES, R>(lds + (j + u) * WORDS,
                                                                     (uint32_t)(base + j + u), d0,
                                                                     best, second);
        }
        for (; j < ncols; ++j)
            search_step<WORDS, NODUPES, R>(lds + j * WORDS, (uint32_t)(base + j), d0, best, second);
    }

    int16_t* __restrict__ out = a.out + (size_t)row * a.out_pitch;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int c0 = col0_base + r * 64;
        if (c0 >= cols) continue;
        const int b = (int)(best[r] & 0xFFFFu);
        const bool dup = NODUPES && ((second[r] >> 16) == (best[r] >> 16));
        int16_t v;
        if (a.out_mode == 0)
            v = dup ? INVALID_I16 : (int16_t)(c0 - b);
        else
            v = dup ? (int16_t)-1 : (int16_t)b;
        out[c0] = v;
    }
}

// Left-right consistency (bicos.hpp:99-106): fwd[c0] = best col1 (or -1), rev[c1] = best
// col0 of the reverse search (or -1).
__global__ __launch_bounds__(256) void consistency_kernel(ConsistencyArgs a) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y;
    if (col >= a.cols) return;
    const int16_t f = a.fwd[(size_t)row * a.cols + col];
    int16_t v = INVALID_I16;
    if (f >= 0) {
        const int rv = a.rev[(size_t)row * a.cols + f];
        if (rv >= 0 && abs(col - rv) <= a.max_lr_diff) v = (int16_t)((col + rv) / 2 - f);
    }
    a.out[(size_t)row * a.out_pitch + col] = v;
}

// ---------------------------------------------------------------------- agree

__device__ __forceinline__ float fma_p(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_p(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float div_p(float a, float b) { return __fdiv_rn(a, b); }
__device__ __forceinline__ double div_p(double a, double b) { return __ddiv_rn(a, b); }
__device__ __forceinline__ float sqrt_p(float a) { return __fsqrt_rn(a); }
__device__ __forceinline__ double sqrt_p(double a) { return __dsqrt_rn(a); }

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

// agree (agree.hpp:53-93) fused with the float conversion of cpu.cpp:88-93 and the NaN
// initialisation of the correlation map (cpu.cpp:78-81): writes every output pixel.
template <typename TIn, typename TPrec>
__global__ __launch_bounds__(256) void agree_kernel(AgreeArgs a) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y;
    if (col >= a.cols) return;
    const size_t o = (size_t)row * a.cols + col;
    int d = a.raw[(size_t)row * a.raw_pitch + col];
    TPrec corr = (TPrec)__builtin_nan("");
    if (d != INVALID_I16) {
        const int idx1 = col - d;
        if (idx1 < 0 || idx1 >= a.cols) {
            d = INVALID_I16;
        } else {
            const TIn* s0 = (const TIn*)a.stack0 + (size_t)row * a.row_pitch;
            const TIn* s1 = (const TIn*)a.stack1 + (size_t)row * a.row_pitch;
            corr = nxcorr_dev<TIn, TPrec>(s0 + col, s1 + idx1, a.plane_pitch, a.n, a.has_minvar,
                                          (TPrec)a.minvar);
            if (corr < (TPrec)a.threshold) d = INVALID_I16;  // NaN passes, as in the reference
        }
    }
    if (a.out_f32)
        ((float*)a.out)[o] = (float)d;
    else
        ((int16_t*)a.out)[o] = (int16_t)d;
    if (a.corrmap) ((TPrec*)a.corrmap)[o] = corr;
}

// agree_subpixel (agree.hpp:95-191). MAXN >= n bounds the per-lane register arrays
// (static indices only; t >= n iterations are skipped by wave-uniform branches). The
// quadratic interpolation is float in both precisions (agree.cuh:221-236).
template <typename TIn, typename TPrec, int MAXN>
__global__ __launch_bounds__(256) void subpixel_kernel(AgreeArgs a) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y;
    if (col >= a.cols) return;
    const size_t o = (size_t)row * a.cols + col;
    const int n = a.n;
    const size_t pp = a.plane_pitch;
    const int d = a.raw[(size_t)row * a.raw_pitch + col];
    const TPrec minvar = (TPrec)a.minvar;
    float out = __builtin_nanf("");
    TPrec corr = (TPrec)__builtin_nan("");
    const int col1 = col - d;
    if (d != INVALID_I16 && col1 >= 0 && col1 < a.cols) {
        const TIn* s0 = (const TIn*)a.stack0 + (size_t)row * a.row_pitch + col;
        const TIn* s1 = (const TIn*)a.stack1 + (size_t)row * a.row_pitch + col1;
        if (col1 == 0 || col1 == a.cols - 1) {
            corr = nxcorr_dev<TIn, TPrec>(s0, s1, pp, n, a.has_minvar, minvar);
            if (!(corr < (TPrec)a.threshold)) out = (float)d;
        } else {
            // left: mean, centred samples and variance are the same for every x
            TPrec D0[MAXN];
            float A[MAXN], B[MAXN], C[MAXN];
            uint32_t s = 0;
#pragma unroll
            for (int t = 0; t < MAXN; ++t)
                if (t < n) {
                    const uint32_t l = ld(s0 + t * pp);
                    D0[t] = (TPrec)l;
                    s += l;
                    const int y0 = (int)ld(s1 - 1 + t * pp);
                    const int y1 = (int)ld(s1 + t * pp);
                    const int y2 = (int)ld(s1 + 1 + t * pp);
                    // 0.5f * ( y0 - 2.0f * y1 + y2) ; 0.5f * (-y0 + y2) ; y1
                    A[t] = 0.5f * (((float)y0 - 2.0f * (float)y1) + (float)y2);
                    B[t] = 0.5f * (float)(-y0 + y2);
                    C[t] = (float)y1;
                }
            const TPrec m0 = div_p((TPrec)s, (TPrec)n);
            TPrec v0 = 0;
#pragma unroll
            for (int t = 0; t < MAXN; ++t)
                if (t < n) {
                    D0[t] = D0[t] - m0;
                    v0 = fma_p(D0[t], D0[t], v0);
                }
            const bool v0_low = a.has_minvar && v0 < minvar;

            float best_x = 0.f;
            TPrec best = -1;
            const float step = a.step;
            for (float x = -1.f; x <= 1.f; x += step) {
                float IV[MAXN];
                uint32_t si = 0;
#pragma unroll
                for (int t = 0; t < MAXN; ++t)
                    if (t < n) {
                        const float ax = A[t] * x;
                        const float v = (ax * x + B[t] * x) + C[t];
                        // (TIn)roundevenf(v): the narrowing wraps through int32
                        const uint32_t iv = (uint32_t)(TIn)(int)__builtin_rintf(v);
                        IV[t] = (float)iv;
                        si += iv;
                    }
                const TPrec m1 = div_p((TPrec)si, (TPrec)n);
                TPrec cov = 0, v1 = 0;
#pragma unroll
                for (int t = 0; t < MAXN; ++t)
                    if (t < n) {
                        const TPrec x1 = (TPrec)IV[t] - m1;
                        cov = fma_p(D0[t], x1, cov);
                        v1 = fma_p(x1, x1, v1);
                    }
                TPrec nxc;
                if (v0_low || (a.has_minvar && v1 < minvar))
                    nxc = -1;
                else
                    nxc = div_p(cov, sqrt_p(v0 * v1));
                if (best < nxc) {
                    best_x = x;
                    best = nxc;
                }
            }
            corr = best;
            if (!(best < (TPrec)a.threshold)) out = (float)d - best_x;
        }
    }
    ((float*)a.out)[o] = out;
    if (a.corrmap) ((TPrec*)a.corrmap)[o] = corr;
}

// ------------------------------------------------------------------- dispatch

template <typename TIn, int WORDS>
hipError_t launch_transform_w(const TransformArgs& a, int mode, hipStream_t st) {
    dim3 grid((a.cols + 255) / 256, a.rows, a.stack1 ? 2 : 1);
    if (mode == 0)
        hipLaunchKernelGGL((transform_kernel<TIn, WORDS, 0>), grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((transform_kernel<TIn, WORDS, 1>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

template <typename TIn>
hipError_t launch_transform_t(const TransformArgs& a, int mode, int words, hipStream_t st) {
    switch (words) {
        case 1: return launch_transform_w<TIn, 1>(a, mode, st);
        case 2: return launch_transform_w<TIn, 2>(a, mode, st);
        case 4: return launch_transform_w<TIn, 4>(a, mode, st);
        case 8: return launch_transform_w<TIn, 8>(a, mode, st);
    }
    return hipErrorInvalidValue;
}

template <int WORDS, bool NODUPES, int R>
hipError_t launch_search_r(const SearchArgs& a, int waves, hipStream_t st) {
    const size_t lds = (size_t)a.chunk * WORDS * 4;
    const int nwg = a.rows * a.tiles_per_row;
    hipLaunchKernelGGL((search_kernel<WORDS, NODUPES, R>), dim3(nwg), dim3(64 * waves), lds, st, a);
    return hipGetLastError();
}

template <int WORDS, bool NODUPES>
hipError_t launch_search_n(const SearchArgs& a, int R, int waves, hipStream_t st) {
    switch (R) {
        case 1: return launch_search_r<WORDS, NODUPES, 1>(a, waves, st);
        case 2: return launch_search_r<WORDS, NODUPES, 2>(a, waves, st);
        case 4: return launch_search_r<WORDS, NODUPES, 4>(a, waves, st);
    }
    return hipErrorInvalidValue;
}

template <int WORDS>
hipError_t launch_search_w(const SearchArgs& a, bool nodupes, int R, int waves, hipStream_t st) {
    return nodupes ? launch_search_n<WORDS, true>(a, R, waves, st)
                   : launch_search_n<WORDS, false>(a, R, waves, st);
}

template <typename TIn, typename TPrec, int MAXN>
hipError_t launch_subpixel_m(const AgreeArgs& a, hipStream_t st) {
    dim3 grid((a.cols + 255) / 256, a.rows);
    hipLaunchKernelGGL((subpixel_kernel<TIn, TPrec, MAXN>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

template <typename TIn, typename TPrec>
hipError_t launch_subpixel_t(const AgreeArgs& a, hipStream_t st) {
    const int n = a.n;
    if (n <= 8) return launch_subpixel_m<TIn, TPrec, 8>(a, st);
    if (n <= 16) return launch_subpixel_m<TIn, TPrec, 16>(a, st);
    if (n <= 24) return launch_subpixel_m<TIn, TPrec, 24>(a, st);
    if (n <= 33) return launch_subpixel_m<TIn, TPrec, 33>(a, st);
    if (n <= 40) return launch_subpixel_m<TIn, TPrec, 40>(a, st);
    if (n <= 48) return launch_subpixel_m<TIn, TPrec, 48>(a, st);
    if (n <= 56) return launch_subpixel_m<TIn, TPrec, 56>(a, st);
    if (n <= 65) return launch_subpixel_m<TIn, TPrec, 65>(a, st);
    return hipErrorInvalidValue;
}

template <typename TIn, typename TPrec>
hipError_t launch_agree_t(const AgreeArgs& a, hipStream_t st) {
    dim3 grid((a.cols + 255) / 256, a.rows);
    hipLaunchKernelGGL((agree_kernel<TIn, TPrec>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace

// ------------------------------------------------------------ public launchers

hipError_t launch_transform(const TransformArgs& a, int depth, int mode, int words, hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    if (mode == 1 && a.n > 16) return hipErrorInvalidValue;
    return depth == 1 ? launch_transform_t<uint8_t>(a, mode, words, st)
                      : launch_transform_t<uint16_t>(a, mode, words, st);
}

SearchGeometry search_geometry(int rows, int cols, int words, int max_lds_bytes) {
    SearchGeometry g;
    // col1 chunk staged per LDS fill: the whole row when it fits
    const int max_chunk = max_lds_bytes / (words * 4);
    g.chunk = cols < max_chunk ? cols : max_chunk;
    // register blocking and waves: enough workgroups to cover 256 CUs several times
    g.waves = 4;
    g.R = 2;
    const long per_wg = 64L * g.waves * g.R;
    long tiles = (cols + per_wg - 1) / per_wg;
    if ((long)rows * tiles < 1024) {
        g.R = 1;
    }
    g.tiles_per_row = (int)((cols + 64L * g.waves * g.R - 1) / (64L * g.waves * g.R));
    return g;
}

hipError_t launch_search(SearchArgs a, const SearchGeometry& g, int words, bool nodupes,
                         hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    a.chunk = g.chunk;
    a.tiles_per_row = g.tiles_per_row;
    switch (words) {
        case 1: return launch_search_w<1>(a, nodupes, g.R, g.waves, st);
        case 2: return launch_search_w<2>(a, nodupes, g.R, g.waves, st);
        case 4: return launch_search_w<4>(a, nodupes, g.R, g.waves, st);
        case 8: return launch_search_w<8>(a, nodupes, g.R, g.waves, st);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_consistency(const ConsistencyArgs& a, hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    dim3 grid((a.cols + 255) / 256, a.rows);
    hipLaunchKernelGGL(consistency_kernel, grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_agree(const AgreeArgs& a, int depth, bool dbl, hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    if (depth == 1)
        return dbl ? launch_agree_t<uint8_t, double>(a, st) : launch_agree_t<uint8_t, float>(a, st);
    return dbl ? launch_agree_t<uint16_t, double>(a, st) : launch_agree_t<uint16_t, float>(a, st);
}

hipError_t launch_subpixel(const AgreeArgs& a, int depth, bool dbl, hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    if (depth == 1)
        return dbl ? launch_subpixel_t<uint8_t, double>(a, st)
                   : launch_subpixel_t<uint8_t, float>(a, st);
    return dbl ? launch_subpixel_t<uint16_t, double>(a, st)
               : launch_subpixel_t<uint16_t, float>(a, st);
}

}  // namespace bicos_hip
