// kernels.hip -- gfx950 (CDNA4) kernels of the BICOS hot path.
//
//   transform_kernel    descriptor_transform  (reference include/impl/cpu/descriptor_transform.hpp:31-138)
//   search16_kernel     bicos Hamming search on the VALU (reference include/impl/cpu/bicos.hpp:29-113;
//                       the default search runs on the matrix cores: search_mx.hip)
//   consistency_kernel  left-right check      (reference include/impl/cpu/bicos.hpp:99-106)
//   agree_kernel        NXC filter            (reference include/impl/cpu/agree.hpp:28-93)
//   (subpixel_kernel, the NXC + quadratic refine of agree.hpp:95-191: subpixel.hpp)
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
#include "nxc.hpp"
#include "stack.hpp"
#include "transform.hpp"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include <type_traits>

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


using nxc::ld;
using nxc::fma_p;
using nxc::div_p;
using nxc::sqrt_p;
using nxc::nxcorr_dev;


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

template <typename TIn, int WORDS, int MAXN, bool EXACT>
__global__ __launch_bounds__(256) void transform_limited_kernel(TransformArgs a) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y;
    const int which = blockIdx.z;
    if (col >= a.cols) return;
    const StackReader<TIn> rd(which ? a.stack1 : a.stack0, a.stack_bytes);
    uint32_t* __restrict__ out = (which ? a.desc1 : a.desc0) + (size_t)row * a.desc_pitch + (size_t)col * WORDS;
    const uint32_t pp = (uint32_t)a.plane_pitch;
    const uint32_t rowoff = (uint32_t)row * (uint32_t)a.row_pitch;
    // EXACT: n == MAXN, so every `t < n` below is a compile-time constant
    uint32_t w[WORDS];
    limited_descriptor<TIn, WORDS, MAXN, EXACT>(rd, (uint32_t)col, rowoff, pp, a.n, a.magic, w);

    if (WORDS % 4 == 0) {
#pragma unroll
        for (int k = 0; k < WORDS; k += 4)
            *(uint4*)(out + k) = make_uint4(w[k], w[k + 1], w[k + 2], w[k + 3]);
    } else if (WORDS == 2) {
        *(uint2*)out = make_uint2(w[0], w[1 % WORDS]);
    } else {
        out[0] = w[0];
    }
}

// FULL transform with the stack size N a template parameter (transform.hpp
// full_descriptor): every bit at a static position. Used when the descriptor width is the
// one the match picks for N (launch_transform_w); transform_kernel<..., 1> otherwise.
template <typename TIn, int WORDS, int N>
__global__ __launch_bounds__(256) void transform_full_kernel(TransformArgs a) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y;
    const int which = blockIdx.z;
    if (col >= a.cols) return;
    const StackReader<TIn> rd(which ? a.stack1 : a.stack0, a.stack_bytes);
    uint32_t* __restrict__ out = (which ? a.desc1 : a.desc0) + (size_t)row * a.desc_pitch + (size_t)col * WORDS;
    uint32_t w[WORDS];
    full_descriptor<TIn, WORDS, N>(rd, (uint32_t)col, (uint32_t)row * (uint32_t)a.row_pitch,
                                   (uint32_t)a.plane_pitch, a.magic, w);
    if (WORDS % 4 == 0) {
#pragma unroll
        for (int k = 0; k < WORDS; k += 4)
            *(uint4*)(out + k) = make_uint4(w[k], w[k + 1], w[k + 2], w[k + 3]);
    } else if (WORDS == 2) {
        *(uint2*)out = make_uint2(w[0], w[1 % WORDS]);
    } else {
        out[0] = w[0];
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

// ---- the VALU search: packed 16-bit keys ------------------------------------------
//
// Measured on MI355X (tools/valu_peak.hip): v_xor/v_and/v_add issue at full rate
// (~72 T lane-op/s) but v_bcnt, v_min, v_med3, v_lshl_or, v_perm and v_pk_*_u16 at half
// rate (~38.5 T). A direct 32-bit-key loop (cost << 16 | col1 per pair, v_med3 + v_min)
// spends 7 half-rate ops per pair for w = 4 (measured 11 % slower; removed in round 2, as
// were two hand-scheduled forms of this loop). Here two col0 share one 32-bit register
// of two 16-bit keys (cost << 8 | col1 within a 256-column tile):
//   r0, r1  = bcnt chains seeded with (col1_local << 8)  -> byte1 = col1, byte0 = cost
//   key     = v_perm_b32(r1, r0)      [r0.b1 r0.b0 | r1.b1 r1.b0]  (1 op / 2 pairs)
//   lo      = v_pk_min_u16(lo, key)   first minimum (lowest col1)  (1 op / 2 pairs)
//   hi      = v_pk_min_u16(hi, key ^ 0x00FF00FF)   last minimum    (1 op + 1 fast xor)
// The minimum is duplicated iff its first and last columns differ. Tiles fold into
// 32-bit keys (cost << 16 | col1). Costs must fit 8 bits: descriptors from the transform
// use <= 254 bits (LIMITED 4n-6 <= 254, FULL n^2-2n+3 <= 227), and bit 255 is masked
// on both sides when the descriptor has 256 bits, so cost <= 255.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}

// The same step in C with an instruction-free asm keeping each bcnt accumulator opaque
// (so the chain is not re-associated into v_add3); the compiler schedules freely.
template <int WORDS>
__device__ __forceinline__ uint32_t ham_seeded(const uint32_t (&a)[WORDS], const uint32_t (&b)[WORDS],
                                               uint32_t seed) {
    uint32_t c = bcnt_acc(a[0] ^ b[0], seed);
#pragma unroll
    for (int k = 1; k < WORDS; ++k) c = bcnt_acc(a[k] ^ b[k], c);
    return c;
}

template <int WORDS, bool NODUPES, int RP>
__device__ __forceinline__ void search16_step(const uint32_t* s, uint32_t seed,
                                              const uint32_t (&d0)[2 * RP][WORDS],
                                              uint32_t (&lo)[RP], uint32_t (&hi)[RP]) {
    uint32_t d1[WORDS];
    lds_fetch<WORDS>(s, d1);
#pragma unroll
    for (int p = 0; p < RP; ++p) {
        const uint32_t r0 = ham_seeded<WORDS>(d0[2 * p], d1, seed);
        const uint32_t r1 = ham_seeded<WORDS>(d0[2 * p + 1], d1, seed);
        const uint32_t key = __builtin_amdgcn_perm(r1, r0, 0x04050001u);
        lo[p] = pk_min_u16(lo[p], key);
        if (NODUPES) hi[p] = pk_min_u16(hi[p], key ^ 0x00FF00FFu);
    }
}

// The VALU search is kept as an independent cross-check of the matrix-core search
// (BICOS_SEARCH=valu; identical results).
template <int WORDS, bool NODUPES, int RP>
__global__ __launch_bounds__(512) void search16_kernel(SearchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int per_xcd = (nwg + 7) / 8;
    int logical = (bid % 8) * per_xcd + bid / 8;
    if (nwg % 8 != 0) logical = bid;
    const int row = logical / a.tiles_per_row;
    const int tile = logical % a.tiles_per_row;

    constexpr int R = 2 * RP;
    // waves = groups x split: the `split` waves of a group hold the same col0 and scan
    // interleaved 256-column tiles of the right row; their minima merge through LDS.
    const int split = a.split;
    const int groups = blockDim.x / 64 / split;
    const int wave = threadIdx.x / 64;
    const int group = wave / split;
    const int seg = wave % split;
    const int lane = threadIdx.x % 64;
    const int cols = a.cols;
    const int col0_base = tile * groups * 64 * R + group * 64 * R + lane;
    const bool idle = col0_base - lane >= cols;  // wave-uniform
    const uint32_t top_mask = WORDS == 8 ? 0x7FFFFFFFu : 0xFFFFFFFFu;

    const uint32_t* __restrict__ row0 = a.desc0 + (size_t)row * a.desc_pitch;
    const uint32_t* __restrict__ row1 = a.desc1 + (size_t)row * a.desc_pitch;

    uint32_t d0[R][WORDS];
    uint32_t glo[R], ghi[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int c0 = col0_base + r * 64;
        const int cc = c0 < cols ? c0 : cols - 1;
        lds_fetch<WORDS>(row0 + (size_t)cc * WORDS, d0[r]);
        d0[r][WORDS - 1] &= top_mask;
        glo[r] = 0xFFFFFFFFu;
        ghi[r] = 0xFFFFFFFFu;
    }

    for (int base = 0; base < cols; base += a.chunk) {
        const int ncols = min(a.chunk, cols - base);
        const int nwords = ncols * WORDS;
        if (base) __syncthreads();
        {
            const uint32_t* src = row1 + (size_t)base * WORDS;
            const int n4 = nwords / 4;
            for (int i = threadIdx.x; i < n4; i += blockDim.x) {
                uint4 v = ((const uint4*)src)[i];
                if (WORDS == 8 && (i & 1)) v.w &= top_mask;
                ((uint4*)lds)[i] = v;
            }
            for (int i = n4 * 4 + threadIdx.x; i < nwords; i += blockDim.x) lds[i] = src[i];
        }
        __syncthreads();

        // a wave whose col0 all lie beyond the image (last tile of a row) has nothing to
        // search: it only helps stage the row (cfg5, 3840 columns: 6 % of the waves)
        for (int t0 = idle ? ncols : seg * 256; t0 < ncols; t0 += 256 * split) {
            const int tn = min(256, ncols - t0);
            uint32_t lo[RP], hi[RP];
#pragma unroll
            for (int p = 0; p < RP; ++p) {
                lo[p] = 0xFFFFFFFFu;
                hi[p] = 0xFFFFFFFFu;
            }
            const uint32_t* tl = lds + t0 * WORDS;
            constexpr int U = WORDS >= 8 ? 4 : 8;
            int j = 0;
            for (; j + U <= tn; j += U) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    search16_step<WORDS, NODUPES, RP>(tl + (j + u) * WORDS,
                                                            (uint32_t)(j + u) << 8, d0, lo, hi);
            }
            for (; j < tn; ++j)
                search16_step<WORDS, NODUPES, RP>(tl + j * WORDS, (uint32_t)j << 8, d0, lo,
                                                        hi);

            // fold the tile's 16-bit keys into 32-bit (cost << 16 | col1) keys
            const uint32_t tb = (uint32_t)(base + t0);
#pragma unroll
            for (int p = 0; p < RP; ++p) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t v = (lo[p] >> (16 * h)) & 0xFFFFu;
                    const uint32_t k = ((v >> 8) << 16) | (tb + (v & 0xFFu));
                    glo[2 * p + h] = min(glo[2 * p + h], k);
                    if (NODUPES) {
                        const uint32_t w = (hi[p] >> (16 * h)) & 0xFFFFu;
                        const uint32_t last = tb + 255u - (w & 0xFFu);
                        const uint32_t kh = ((w >> 8) << 16) | (0xFFFFu - last);
                        ghi[2 * p + h] = min(ghi[2 * p + h], kh);
                    }
                }
            }
        }
    }

    if (split > 1) {
        // merge the segments' minima (min of disjoint col1 ranges is exact)
        __syncthreads();
        uint32_t* m = lds;  // the row stage is dead now
        const int slot = (group * 64 + lane) * R;
        if (seg > 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                m[((seg - 1) * groups * 64 * R + slot + r) * 2] = glo[r];
                m[((seg - 1) * groups * 64 * R + slot + r) * 2 + 1] = ghi[r];
            }
        }
        __syncthreads();
        if (seg > 0) return;
        for (int q = 0; q < split - 1; ++q)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                glo[r] = min(glo[r], m[(q * groups * 64 * R + slot + r) * 2]);
                ghi[r] = min(ghi[r], m[(q * groups * 64 * R + slot + r) * 2 + 1]);
            }
    }

    int16_t* __restrict__ out = a.out + (size_t)row * a.out_pitch;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int c0 = col0_base + r * 64;
        if (c0 >= cols) continue;
        const int first = (int)(glo[r] & 0xFFFFu);
        const bool dup = NODUPES && (int)(0xFFFFu - (ghi[r] & 0xFFFFu)) != first;
        int16_t v;
        if (a.out_mode == 0)
            v = dup ? INVALID_I16 : (int16_t)(c0 - first);
        else
            v = dup ? (int16_t)-1 : (int16_t)first;
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

// fma_p / div_p / sqrt_p (IEEE, correctly rounded): nxc.hpp


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


// agree with the 2n samples loaded once into registers (MAXN >= n), the same arithmetic
// and output contract as agree_kernel.
template <typename TIn, typename TPrec, int MAXN, bool EXACT>
__global__ __launch_bounds__(256) void agree_reg_kernel(AgreeArgs a) {
    int tile, row;
    xcd_rows(tile, row);
    const int col = tile * 256 + threadIdx.x;
    if (col >= a.cols) return;
    const size_t o = (size_t)row * a.cols + col;
    int d = a.raw[(size_t)row * a.raw_pitch + col];
    // Straight-line loads: the left samples do not depend on d, so they are issued while
    // the disparity load is in flight; the right ones read column col for pixels without
    // a match (cached, discarded). Branching on d first serialised the two loads per wave
    // (the kernel was latency-bound at 3.2 TB/s; a plain planar read runs at 6.8).
    const int idx1 = col - d;
    const bool inb = d != INVALID_I16 && idx1 >= 0 && idx1 < a.cols;
    const int n = EXACT ? MAXN : a.n;
    const size_t pp = a.plane_pitch;
    const StackReader<TIn> rd0(a.stack0, a.stack_bytes), rd1(a.stack1, a.stack_bytes);
    const uint32_t rowoff = (uint32_t)row * (uint32_t)a.row_pitch;
    uint32_t l[MAXN], r[MAXN];
    uint32_t sl = 0, sr = 0;
#pragma unroll
    for (int t = 0; t < MAXN; ++t)
        if (t < n) l[t] = rd0((uint32_t)col, rowoff + (uint32_t)(t * pp));
    const uint32_t c1 = inb ? (uint32_t)idx1 : (uint32_t)col;
#pragma unroll
    for (int t = 0; t < MAXN; ++t)
        if (t < n) r[t] = rd1(c1, rowoff + (uint32_t)(t * pp));
#pragma unroll
    for (int t = 0; t < MAXN; ++t)
        if (t < n) {
            sl += l[t];
            sr += r[t];
        }
    TPrec corr = (TPrec)__builtin_nan("");
    if (inb) {
        const TPrec m0 = div_p((TPrec)sl, (TPrec)n);
        const TPrec m1 = div_p((TPrec)sr, (TPrec)n);
        TPrec cov = 0, v0 = 0, v1 = 0;
#pragma unroll
        for (int t = 0; t < MAXN; ++t)
            if (t < n) {
                const TPrec x0 = (TPrec)l[t] - m0;
                const TPrec x1 = (TPrec)r[t] - m1;
                cov = fma_p(x0, x1, cov);
                v0 = fma_p(x0, x0, v0);
                v1 = fma_p(x1, x1, v1);
            }
        if (a.has_minvar && (v0 < (TPrec)a.minvar || v1 < (TPrec)a.minvar))
            corr = (TPrec)-1;
        else
            corr = div_p(cov, sqrt_p(v0 * v1));
        if (corr < (TPrec)a.threshold) d = INVALID_I16;  // NaN passes, as in the reference
    } else {
        d = INVALID_I16;
    }
    if (a.out_f32)
        ((float*)a.out)[o] = (float)d;
    else
        ((int16_t*)a.out)[o] = (int16_t)d;
    if (a.corrmap) ((TPrec*)a.corrmap)[o] = corr;
}

// agree_reg_kernel with the left samples staged through LDS: the workgroup's 256-column
// tile of all n left planes is fetched with dword loads (one wave-uniform plane per load:
// 64 lanes x 4 B = one 256-byte plane row of 8-bit data), so a lane keeps only its n right
// samples in registers (~55 VGPRs at n = 33: 8 waves/SIMD instead of 4). The right
// samples are gathered at col - d as before; the left loads, the disparity load and the
// right gathers are all in flight together. Requires 4-byte aligned stacks, row and
// plane pitches (checked on the host; agree_reg_kernel otherwise). Same contract and
// results as agree_reg_kernel.
//
// CONS: Consistency's left-right check (consistency_kernel, reference bicos.hpp:99-106) in
// the same launch -- the pixel's disparity comes from the forward / reverse search results
// (a.fwd, a.rev) instead of a.raw: one launch and one int16 map round trip fewer per frame
// (cfg4). The forward result and the reverse gather at it are loaded first, then the left
// tile, so the right gathers wait on both search results but not on the tile.
template <typename TIn, typename TPrec, int MAXN, bool EXACT, bool CONS = false>
__global__ __launch_bounds__(256) void agree_lds_kernel(AgreeArgs a) {
    constexpr int DW = 64 * (int)sizeof(TIn);  // dwords per plane of a 256-column tile
    constexpr int WPP = 256 / DW;              // planes per pass of the workgroup
    constexpr int PASSES = (MAXN + WPP - 1) / WPP;
    __shared__ uint32_t tile_l[MAXN * DW];
    int tile, row;
    xcd_rows(tile, row);
    const int col0 = tile * 256;
    const int col = col0 + (int)threadIdx.x;
    const bool live = col < a.cols;
    const int n = EXACT ? MAXN : a.n;
    const uint32_t pp = (uint32_t)a.plane_pitch;
    const uint32_t rowoff = (uint32_t)row * (uint32_t)a.row_pitch;
    int d = INVALID_I16;
    if constexpr (CONS) {
        // unguarded loads (see below): an invalid or dead pixel reads column 0
        const size_t ro = (size_t)row * a.cols;
        const int f = a.fwd[ro + (live ? col : 0)];
        const int rv = a.rev[ro + (f >= 0 ? f : 0)];
        if (live && f >= 0 && rv >= 0 && abs(col - rv) <= a.max_lr_diff)
            d = (int)(int16_t)((col + rv) / 2 - f);
    } else {
        d = live ? (int)a.raw[(size_t)row * a.raw_pitch + col] : INVALID_I16;
    }
    // the range covers whole dwords: with a padded pitch and cols % 4 != 0 the stack's last
    // pixel shares a dword with up to 3 bytes past it, and a dword reaching past
    // num_records reads as 0 -- the last row's last pixels of plane n-1 came in as 0
    // (tests/test_gpu_parity.py::test_padded_pitch_odd_width). Those bytes lie in the same
    // aligned dword as valid pixels (base 4-aligned), so reading them cannot fault.
    const uint32_t range = a.stack_bytes > 0xFFFFFFFCu ? 0xFFFFFFFFu : (a.stack_bytes + 3u) & ~3u;
    const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(a.stack0), (short)0, (int)range, 0x00020000);
    // left tile loads: pass j, wave-uniform plane p = j * WPP + tid / DW, dword tid % DW
    const int p0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x / DW);
    const uint32_t lane_b = (uint32_t)col0 * sizeof(TIn) + 4u * (threadIdx.x % DW);
    uint32_t w[PASSES];
#pragma unroll
    for (int j = 0; j < PASSES; ++j) {
        // unconditional (planes past n re-read plane n-1, not stored): a guarded load
        // ends in a control-flow join where the waitcnt pass waits for every load
        const int p = min(j * WPP + p0, n - 1);
        w[j] = __builtin_amdgcn_raw_buffer_load_b32(
            r0, lane_b, (rowoff + (uint32_t)p * pp) * (uint32_t)sizeof(TIn), 0);
    }
    const int idx1 = col - d;
    const bool inb = live && d != INVALID_I16 && idx1 >= 0 && idx1 < a.cols;
    const uint32_t c1 = inb ? (uint32_t)idx1 : 0u;
    const StackReader<TIn> rd1(a.stack1, a.stack_bytes);
    uint32_t r[MAXN];
#pragma unroll
    for (int t = 0; t < MAXN; ++t)  // unconditional as above (slots past n: plane n-1)
        r[t] = rd1(c1, rowoff + (uint32_t)min(t, n - 1) * pp);
#pragma unroll
    for (int j = 0; j < PASSES; ++j) {
        const int p = j * WPP + p0;
        if (p < n) tile_l[p * DW + threadIdx.x % DW] = w[j];
    }
    __syncthreads();
    if (!live) return;
    const TIn* lt = (const TIn*)tile_l + threadIdx.x;  // plane t at lt[t * 256]
    const size_t o = (size_t)row * a.cols + col;
    TPrec corr = (TPrec)__builtin_nan("");
    if (inb) {
        uint32_t sl = 0, sr = 0;
#pragma unroll
        for (int t = 0; t < MAXN; ++t)
            if (t < n) {
                sl += lt[t * 256];
                sr += r[t];
                // LDS reads next to their use: hoisted, they cost n more VGPRs
                if ((t & 7) == 7) __builtin_amdgcn_sched_barrier(0);
            }
        // re-read the left samples from LDS in the second pass instead of holding them
        asm volatile("" ::: "memory");
        const TPrec m0 = div_p((TPrec)sl, (TPrec)n);
        const TPrec m1 = div_p((TPrec)sr, (TPrec)n);
        TPrec cov = 0, v0 = 0, v1 = 0;
#pragma unroll
        for (int t = 0; t < MAXN; ++t)
            if (t < n) {
                const TPrec x0 = (TPrec)(uint32_t)lt[t * 256] - m0;
                const TPrec x1 = (TPrec)r[t] - m1;
                cov = fma_p(x0, x1, cov);
                v0 = fma_p(x0, x0, v0);
                v1 = fma_p(x1, x1, v1);
                if ((t & 7) == 7) __builtin_amdgcn_sched_barrier(0);
            }
        if (a.has_minvar && (v0 < (TPrec)a.minvar || v1 < (TPrec)a.minvar))
            corr = (TPrec)-1;
        else
            corr = div_p(cov, sqrt_p(v0 * v1));
        if (corr < (TPrec)a.threshold) d = INVALID_I16;  // NaN passes, as in the reference
    } else {
        d = INVALID_I16;
    }
    if (a.out_f32)
        ((float*)a.out)[o] = (float)d;
    else
        ((int16_t*)a.out)[o] = (int16_t)d;
    if (a.corrmap) ((TPrec*)a.corrmap)[o] = corr;
}

// ------------------------------------------------------------------- dispatch

template <typename TIn, int WORDS, int MAXN>
hipError_t launch_tl(const TransformArgs& a, dim3 grid, hipStream_t st) {
    if (a.n == MAXN)
        hipLaunchKernelGGL((transform_limited_kernel<TIn, WORDS, MAXN, true>), grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((transform_limited_kernel<TIn, WORDS, MAXN, false>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

template <typename TIn, int WORDS>
hipError_t launch_transform_w(const TransformArgs& a, int mode, hipStream_t st) {
    dim3 grid((a.cols + 255) / 256, a.rows, a.stack1 ? 2 : 1);
    if (mode == 0) {
        // descriptor width bounds n: 32 bits -> n <= 9, 64 -> 17, 128 -> 33, 256 -> 65
        const int n = a.n;
        if constexpr (WORDS == 1) return launch_tl<TIn, WORDS, 9>(a, grid, st);
        else if constexpr (WORDS == 2) return n <= 12 ? launch_tl<TIn, WORDS, 12>(a, grid, st)
                                                      : launch_tl<TIn, WORDS, 17>(a, grid, st);
        else if constexpr (WORDS == 4) return n <= 24 ? launch_tl<TIn, WORDS, 24>(a, grid, st)
                                                      : launch_tl<TIn, WORDS, 33>(a, grid, st);
        else if (n <= 40) return launch_tl<TIn, WORDS, 40>(a, grid, st);
        else if (n <= 48) return launch_tl<TIn, WORDS, 48>(a, grid, st);
        else return launch_tl<TIn, WORDS, 65>(a, grid, st);
    }
    // FULL: n^2 - 2n + 3 bits; the static kernel for the width the match uses for n
#define BICOS_FULL_N(N)                                                                   \
    case N:                                                                               \
        if constexpr (WORDS == (N * N - 2 * N + 3 <= 32 ? 1 : N * N - 2 * N + 3 <= 64 ? 2  \
                                : N * N - 2 * N + 3 <= 128 ? 4 : 8)) {                     \
            hipLaunchKernelGGL((transform_full_kernel<TIn, WORDS, N>), grid, dim3(256), 0, st, a); \
            return hipGetLastError();                                                     \
        }                                                                                 \
        break;
    switch (a.n) {
        BICOS_FULL_N(2) BICOS_FULL_N(3) BICOS_FULL_N(4) BICOS_FULL_N(5) BICOS_FULL_N(6)
        BICOS_FULL_N(7) BICOS_FULL_N(8) BICOS_FULL_N(9) BICOS_FULL_N(10) BICOS_FULL_N(11)
        BICOS_FULL_N(12) BICOS_FULL_N(13) BICOS_FULL_N(14) BICOS_FULL_N(15) BICOS_FULL_N(16)
    }
#undef BICOS_FULL_N
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

template <int WORDS, bool NODUPES, int RP>
hipError_t launch_search16_r(const SearchArgs& a, int waves, hipStream_t st) {
    const size_t stage = (size_t)a.chunk * WORDS * 4;
    const size_t merge = a.split > 1 ? (size_t)(waves / a.split) * 64 * (2 * RP) * 8 * (a.split - 1) : 0;
    const size_t lds = stage > merge ? stage : merge;
    const int nwg = a.rows * a.tiles_per_row;
    hipLaunchKernelGGL((search16_kernel<WORDS, NODUPES, RP>), dim3(nwg), dim3(64 * waves), lds, st, a);
    return hipGetLastError();
}

template <int WORDS, bool NODUPES>
hipError_t launch_search_n(const SearchArgs& a, const SearchGeometry& g, hipStream_t st) {
    switch (g.R) {
        case 2: return launch_search16_r<WORDS, NODUPES, 1>(a, g.waves, st);
        case 4: return launch_search16_r<WORDS, NODUPES, 2>(a, g.waves, st);
    }
    return hipErrorInvalidValue;
}

template <int WORDS>
hipError_t launch_search_w(const SearchArgs& a, bool nodupes, const SearchGeometry& g,
                           hipStream_t st) {
    return nodupes ? launch_search_n<WORDS, true>(a, g, st) : launch_search_n<WORDS, false>(a, g, st);
}


template <typename TIn, typename TPrec, int MAXN>
hipError_t launch_agree_m(const AgreeArgs& a, hipStream_t st) {
    dim3 grid((a.cols + 255) / 256, a.rows);
    // left tile through LDS when the dword loads are aligned
    const size_t sz = sizeof(TIn);
    const bool aligned = ((uintptr_t)a.stack0 % 4 == 0) && (a.row_pitch * sz) % 4 == 0 &&
                         (a.plane_pitch * sz) % 4 == 0;
    if (a.fwd) {  // Consistency's check in the agree: the LDS kernel only (engine.cpp plan)
        if (!aligned || !a.rev) return hipErrorInvalidValue;
        hipLaunchKernelGGL((agree_lds_kernel<TIn, TPrec, MAXN, false, true>), grid, dim3(256), 0, st, a);
        return hipGetLastError();
    }
    if (aligned) {
        // runtime n even for an exact bucket: with a constant n the compiler front-loads
        // the conversions and doubles the VGPRs (49 -> 100 at n = 33)
        hipLaunchKernelGGL((agree_lds_kernel<TIn, TPrec, MAXN, false>), grid, dim3(256), 0, st, a);
        return hipGetLastError();
    }
    if (a.n == MAXN)
        hipLaunchKernelGGL((agree_reg_kernel<TIn, TPrec, MAXN, true>), grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((agree_reg_kernel<TIn, TPrec, MAXN, false>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

template <typename TIn, typename TPrec>
hipError_t launch_agree_t(const AgreeArgs& a, hipStream_t st) {
    const int n = a.n;
    if (n <= 8) return launch_agree_m<TIn, TPrec, 8>(a, st);
    if (n <= 16) return launch_agree_m<TIn, TPrec, 16>(a, st);
    if (n <= 24) return launch_agree_m<TIn, TPrec, 24>(a, st);
    if (n <= 33) return launch_agree_m<TIn, TPrec, 33>(a, st);
    if (n <= 40) return launch_agree_m<TIn, TPrec, 40>(a, st);
    if (n <= 48) return launch_agree_m<TIn, TPrec, 48>(a, st);
    if (n <= 65) return launch_agree_m<TIn, TPrec, 65>(a, st);
    // beyond the descriptor limit only the stage API can get here: generic kernel
    if (a.fwd) return hipErrorInvalidValue;
    dim3 grid((a.cols + 255) / 256, a.rows);
    hipLaunchKernelGGL((agree_kernel<TIn, TPrec>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace

// ------------------------------------------------------------ public launchers

hipError_t launch_transform(TransformArgs a, int depth, int mode, int words, hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    if (mode == 1 && a.n > 16) return hipErrorInvalidValue;
    if (a.n < 2) return hipErrorInvalidValue;
    a.magic = (uint32_t)((0x100000000ull + (uint64_t)a.n - 1) / (uint64_t)a.n);
    return depth == 1 ? launch_transform_t<uint8_t>(a, mode, words, st)
                      : launch_transform_t<uint16_t>(a, mode, words, st);
}

SearchGeometry search_geometry(int rows, int cols, int words, int max_lds_bytes, int variant,
                               int R, int waves, int split, int cus, int extra_col_bytes) {
    SearchGeometry g;
    (void)variant;  // one VALU search remains: packed 16-bit keys (variant 16)
    g.variant = 16;
    // col1 chunk staged per LDS fill: the whole row when it fits
    const int max_chunk = max_lds_bytes / (words * 4 + extra_col_bytes);
    g.chunk = cols < max_chunk ? cols : max_chunk;
    // 8 waves per workgroup: the row stage (<= 64 KiB) caps resident workgroups per CU,
    // so wide workgroups are what fill the 32 wave slots (measured: 4 waves -1 %, 2 waves
    // +40 % time at cfg2)
    g.waves = waves ? waves : 8;
    g.R = R == 4 ? 4 : 2;
    if (split) {
        g.split = split;
    } else {
        // Split the col1 scan across waves so the grid fills whole "rounds" of resident
        // waves (CUs x 32): a round that is only partly filled idles the rest of the chip
        // (192-row bands, 8 GPUs: 1.5 rounds at split 4 vs 3.0 at split 8).
        const long base = (long)rows * ((cols + 64L * g.R - 1) / (64L * g.R));
        const int tiles256 = (cols + 255) / 256;
        const double slots = (double)(cus > 0 ? cus : 256) * 32.0;
        double best = -1.0;
        g.split = 1;
        for (int sp = 1; sp <= 8; sp *= 2) {
            if (sp > 1 && (tiles256 < sp || g.waves % sp)) break;
            const double rounds = (double)(base * sp) / slots;
            const double fill = rounds / __builtin_ceil(rounds);
            // prefer a full last round, then up to 3 rounds in flight, then a smaller split
            const double score = fill + 0.1 * (rounds < 3.0 ? rounds : 3.0) / 3.0 -
                                 0.005 * (double)__builtin_ctz(sp);
            if (score > best + 1e-9) {
                best = score;
                g.split = sp;
            }
        }
    }
    const long per_wg = 64L * (g.waves / g.split) * g.R;
    g.tiles_per_row = (int)((cols + per_wg - 1) / per_wg);
    return g;
}

hipError_t launch_search(SearchArgs a, const SearchGeometry& g, int words, bool nodupes,
                         hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    a.chunk = g.chunk;
    a.tiles_per_row = g.tiles_per_row;
    a.split = g.split;
    if (g.waves % g.split) return hipErrorInvalidValue;
    switch (words) {
        case 1: return launch_search_w<1>(a, nodupes, g, st);
        case 2: return launch_search_w<2>(a, nodupes, g, st);
        case 4: return launch_search_w<4>(a, nodupes, g, st);
        case 8: return launch_search_w<8>(a, nodupes, g, st);
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

}  // namespace bicos_hip
