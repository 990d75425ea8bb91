// search_mx.hip -- the bicos Hamming search (reference include/impl/cpu/bicos.hpp:50-113) on
// the gfx950 matrix cores.
//
// Why a matrix core can do an exact Hamming search. With a = bits of the left (col0)
// descriptor and b = bits of the right (col1) descriptor,
//     ham(a, b) = sum_k a_k + b_k - 2 a_k b_k = |a| + sum_k b_k (1 - 2 a_k).
// |a| is constant over a row scan, so argmin_col1 ham = argmin_col1 x with
//     x(col0, col1) = sum_k B[k][col0] * A[col1][k],  A = b in {0, 1},  B = 1 - 2a in {+1, -1},
// a plain matrix product with K = descriptor bits. Both operands are exact FP4 (e2m1: 0, 1.0,
// -1.0), so one v_mfma_f32_32x32x64_f8f6f4 (FP4 x FP4 -> f32, 32 cycles per SIMD) evaluates
// 32 x 32 pairs x 64 bits; partial sums are small integers, exact in f32.
//
// The argmin key rides in the accumulator input: C[col1][col0] = 256 + col1 * 2^-15, so
//     D1 = A * B + C = 256 + x + col1 * 2^-15
// exactly (|x| <= 255, col1 < 32768: 24 significant bits at most; bit 255 of 256-bit
// descriptors is masked on both sides, as in the VALU search -- transform descriptors use
// at most 254 bits). D1 is positive, so its bit
// pattern orders like the float; min over col1 of bits(D1) picks the smallest x and, among
// equal x, the lowest col1 -- the reference's strict '<' scan (bicos.hpp:56-66). For
// NoDuplicates the same MFMA with the A operand negated gives D2 = 256 - x + col1 * 2^-15,
// whose maximum is the HIGHEST col1 at the minimum cost; the minimum is duplicated iff the
// two columns differ (bicos.hpp:58-73). Per pair the VALU does half a v_min3_u32 (and half a
// v_max3_u32): the xor / popcount work is gone from the vector pipe.
//
// Layout: a workgroup = one row x a range of WAVES*T*32 col0; each wave
// keeps T tiles of 32 left descriptors as B fragments in registers (lane l: col0 = 32t +
// (l & 31), descriptor word 2s + (l >> 5) of K-step s, one bit per FP4 nibble). The right
// row is expanded chunk by chunk into LDS as [word][col1] 16-byte FP4 fragments (one bit
// per nibble, 0 or 1.0), so the A fragment of (block, K-step) is ONE conflict-free
// ds_read_b128 per lane. Accumulator map (32x32 shapes): lane l, register r holds row
// (r & 3) + 8 (r >> 2) + 4 (l >> 5) (= col1 in the block) and column l & 31 (= col0).
#include "kernels.hpp"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bicos_hip {

namespace {

constexpr int16_t INVALID_I16 = -32768;

typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr float KEY_BIAS = 256.f;
constexpr float KEY_EPS = 1.f / 32768.f;  // col1 * 2^-15
constexpr float KEY_PAD = 1.0e30f;        // C of columns beyond the image (A = 0 there)

// nibble p of the result = bit p of `b` (b < 256): 1 -> 0x1
__device__ __forceinline__ uint32_t spread8(uint32_t b) {
    uint32_t t = (b | (b << 12)) & 0x000F000Fu;
    t = (t | (t << 6)) & 0x03030303u;
    return (t | (t << 3)) & 0x11111111u;
}

// 32 descriptor bits -> 32 FP4 elements (element 8q + p = nibble p of dword q = bit 8q + p)
__device__ __forceinline__ v4i expand_bits(uint32_t x) {
    v4i r;
    r[0] = (int)spread8(x & 0xFFu);
    r[1] = (int)spread8((x >> 8) & 0xFFu);
    r[2] = (int)spread8((x >> 16) & 0xFFu);
    r[3] = (int)spread8(x >> 24);
    return r;
}

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
    return min(min(a, b), c);
}
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) {
    return max(max(a, b), c);
}

__device__ __forceinline__ v16f mfma_fp4(v4i a, v4i b, v16f c) {
    const v8i a8 = {a[0], a[1], a[2], a[3], 0, 0, 0, 0};
    const v8i b8 = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    // cbsz = blgp = 4: both operands FP4 e2m1; zero scales = the unscaled instruction
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 0, 0, 0);
}

__device__ __forceinline__ uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }

// col1 encoded in a key (D1 or D2 bits): key - 256 = +-x + col1 * 2^-15, x integer
__device__ __forceinline__ int key_col(uint32_t key) {
    const float v = bitsf(key) - KEY_BIAS;  // exact
    return (int)((v - floorf(v)) * 32768.f);
}

template <int WORDS, bool NODUPES, int T>
__global__ __launch_bounds__(512) void search_mx_kernel(SearchArgs a) {
    constexpr int KS = WORDS >= 2 ? WORDS / 2 : 1;  // 64-bit K-steps
    constexpr int WL = 2 * KS;                      // LDS word slots per col1 (W=1: 1 pad)
    extern __shared__ __attribute__((aligned(16))) v4i lds_mx[];  // [WL][chunk]

    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    // XCD-aware order: the tiles of one row on one XCD (shared right row in its L2)
    const int per_xcd = (nwg + 7) / 8;
    int logical = (bid % 8) * per_xcd + bid / 8;
    if (nwg % 8 != 0) logical = bid;
    const int row = logical / a.tiles_per_row;
    const int tile = logical % a.tiles_per_row;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    const int j = lane & 31;
    const int cols = a.cols;
    const int chunk = a.chunk;
    const int waves = blockDim.x >> 6;
    const int c0_wave = (tile * waves + wave) * (T * 32);

    const uint32_t* __restrict__ row0 = a.desc0 + (size_t)row * a.desc_pitch;
    const uint32_t* __restrict__ row1 = a.desc1 + (size_t)row * a.desc_pitch;

    // B fragments: +1 (0x2) where the left bit is 0, -1 (0xA) where it is 1
    v4i bf[T][KS];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int c0 = c0_wave + 32 * t + j;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int w = 2 * s + h;
            uint32_t x = 0;
            if (c0 < cols && w < WORDS) x = row0[(size_t)c0 * WORDS + w];
            if (WORDS == 8 && w == 7) x &= 0x7FFFFFFFu;  // bit 255 masked (see below)
            const v4i e = expand_bits(x);
#pragma unroll
            for (int q = 0; q < 4; ++q) bf[t][s][q] = (int)(0x22222222u | ((uint32_t)e[q] << 3));
        }
    }

    uint32_t m1[T], m2[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        m1[t] = 0xFFFFFFFFu;
        m2[t] = 0u;
    }

    // row offset of accumulator register r in this lane half
    auto rrow = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };

    // one 32-col1 block against the wave's T tiles
    auto block = [&](const v4i* af, const v16f& c1, const v16f& c2) {
        v4i an[KS];
        if constexpr (NODUPES) {
#pragma unroll
            for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int q = 0; q < 4; ++q) an[s][q] = af[s][q] | (af[s][q] << 2);  // 1.0 -> -1.0
        }
#pragma unroll
        for (int t = 0; t < T; ++t) {
            v16f d = mfma_fp4(af[0], bf[t][0], c1);
#pragma unroll
            for (int s = 1; s < KS; ++s) d = mfma_fp4(af[s], bf[t][s], d);
            uint32_t m = m1[t];
#pragma unroll
            for (int r = 0; r < 16; r += 2) m = umin3(m, fbits(d[r]), fbits(d[r + 1]));
            m1[t] = m;
            if constexpr (NODUPES) {
                v16f e = mfma_fp4(an[0], bf[t][0], c2);
#pragma unroll
                for (int s = 1; s < KS; ++s) e = mfma_fp4(an[s], bf[t][s], e);
                uint32_t M = m2[t];
#pragma unroll
                for (int r = 0; r < 16; r += 2) M = umax3(M, fbits(e[r]), fbits(e[r + 1]));
                m2[t] = M;
            }
        }
    };

    const bool idle = c0_wave >= cols;  // wave-uniform; still joins the barriers
    for (int base = 0; base < cols; base += chunk) {
        const int ncols = min(chunk, cols - base);
        if (base) __syncthreads();
        // expand the chunk's right descriptors: one col1 per thread, all its words
        for (int c = threadIdx.x; c < chunk; c += blockDim.x) {
            const int c1 = base + c;
#pragma unroll
            for (int w = 0; w < WL; ++w) {
                uint32_t x = 0;
                if (c1 < cols && w < WORDS) x = row1[(size_t)c1 * WORDS + w];
                if (WORDS == 8 && w == 7) x &= 0x7FFFFFFFu;
                const v4i e = expand_bits(x);
                v4i v;
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = e[q] << 1;  // 0x1 -> 0x2 (1.0)
                lds_mx[w * chunk + c] = v;
            }
        }
        __syncthreads();
        if (idle) continue;

        v16f cc;
#pragma unroll
        for (int r = 0; r < 16; ++r) cc[r] = KEY_BIAS + (float)(base + rrow(r)) * KEY_EPS;
        const int full = ncols / 32;
        for (int b = 0; b < full; ++b) {
            v4i af[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s) af[s] = lds_mx[(2 * s + h) * chunk + 32 * b + j];
            block(af, cc, cc);
#pragma unroll
            for (int r = 0; r < 16; ++r) cc[r] += 32.f * KEY_EPS;  // exact (< 512)
        }
        if (ncols % 32) {
            // columns beyond the image: A = 0 there, so D1 = KEY_PAD, D2 = 0 never win
            const int b = full;
            v4i af[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s) af[s] = lds_mx[(2 * s + h) * chunk + 32 * b + j];
            v16f c1, c2;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const bool in = 32 * b + rrow(r) < ncols;
                c1[r] = in ? cc[r] : KEY_PAD;
                c2[r] = in ? cc[r] : 0.f;
            }
            block(af, c1, c2);
        }
    }
    if (idle) return;

    // the two lane halves hold the even / odd 4-row groups of every block
#pragma unroll
    for (int t = 0; t < T; ++t) {
        m1[t] = min(m1[t], (uint32_t)__shfl_xor((int)m1[t], 32));
        if constexpr (NODUPES) m2[t] = max(m2[t], (uint32_t)__shfl_xor((int)m2[t], 32));
    }
    int16_t* out = a.out + (size_t)row * a.out_pitch;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        if ((t & 1) != h) continue;  // half 0 writes even tiles, half 1 odd tiles
        const int c0 = c0_wave + 32 * t + j;
        if (c0 >= cols) continue;
        const int best = key_col(m1[t]);
        bool ok = true;
        if constexpr (NODUPES) ok = key_col(m2[t]) == best;
        int16_t v;
        if (a.out_mode == 0)
            v = ok ? (int16_t)(c0 - best) : INVALID_I16;
        else
            v = ok ? (int16_t)best : (int16_t)-1;
        out[c0] = v;
    }
}

template <int WORDS, bool NODUPES, int T>
hipError_t launch_mx(const SearchArgs& a, int waves, hipStream_t st) {
    constexpr int WL = WORDS >= 2 ? WORDS : 2;
    const size_t lds = (size_t)WL * a.chunk * 16;
    const auto kern = search_mx_kernel<WORDS, NODUPES, T>;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void*)kern,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(a.rows * a.tiles_per_row), dim3(64 * waves), lds, st, a);
    return hipGetLastError();
}

template <int WORDS, bool NODUPES>
hipError_t launch_mx_t(const SearchArgs& a, const MxGeometry& g, hipStream_t st) {
    switch (g.T) {
        case 2: return launch_mx<WORDS, NODUPES, 2>(a, g.waves, st);
        case 4: return launch_mx<WORDS, NODUPES, 4>(a, g.waves, st);
        case 8: return launch_mx<WORDS, NODUPES, 8>(a, g.waves, st);
    }
    return hipErrorInvalidValue;
}

template <int WORDS>
hipError_t launch_mx_w(const SearchArgs& a, const MxGeometry& g, bool nodupes, hipStream_t st) {
    return nodupes ? launch_mx_t<WORDS, true>(a, g, st) : launch_mx_t<WORDS, false>(a, g, st);
}

}  // namespace

MxGeometry search_mx_geometry(int rows, int cols, int words, int lds_bytes, int T, int waves,
                              int cus) {
    MxGeometry g;
    const int wl = words >= 2 ? words : 2;
    // LDS chunk of expanded right descriptors (16 B per word per col1), multiple of 32
    int chunk = lds_bytes / (wl * 16);
    chunk &= ~31;
    if (chunk < 32) chunk = 32;
    const int cols32 = (cols + 31) & ~31;
    g.chunk = cols32 < chunk ? cols32 : chunk;
    g.waves = waves ? waves : 8;
    if (T) {
        g.T = T;
    } else {
        // the largest T (fewest right-row expansions per row) that still gives every CU
        // about two workgroups
        g.T = 2;
        for (int t = 8; t >= 2; t /= 2) {
            const long per_wg = 32L * g.waves * t;
            const long nwg = (long)rows * ((cols + per_wg - 1) / per_wg);
            if (nwg >= 2L * (cus > 0 ? cus : 256)) {
                g.T = t;
                break;
            }
        }
    }
    const long per_wg = 32L * g.waves * g.T;
    g.tiles_per_row = (int)((cols + per_wg - 1) / per_wg);
    return g;
}

hipError_t launch_search_mx(SearchArgs a, const MxGeometry& g, int words, bool nodupes,
                            hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    if (a.cols > 32767 || g.chunk < 32 || (g.chunk & 31) || g.waves < 1 || g.waves > 8)
        return hipErrorInvalidValue;
    a.chunk = g.chunk;
    a.tiles_per_row = g.tiles_per_row;
    switch (words) {
        case 1: return launch_mx_w<1>(a, g, nodupes, st);
        case 2: return launch_mx_w<2>(a, g, nodupes, st);
        case 4: return launch_mx_w<4>(a, g, nodupes, st);
        case 8: return launch_mx_w<8>(a, g, nodupes, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace bicos_hip
