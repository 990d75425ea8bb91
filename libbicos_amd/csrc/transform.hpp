// transform.hpp -- the descriptor of one pixel, LIMITED (reference
// include/impl/cpu/descriptor_transform.hpp:31-73, limited_descriptor) and FULL with the
// stack size static (descriptor_transform.hpp:75-123, full_descriptor), used by
// transform_limited_kernel / transform_full_kernel in kernels.hip.
#pragma once

#include "stack.hpp"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bicos_hip {
namespace {

// LIMITED transform, one pixel per lane, the n samples held in registers (MAXN >= n bounds
// the static arrays; slots t >= n are skipped by wave-uniform branches).
//
// Bits are pushed MSB-first into `cur` with v_cmp (-> an SGPR lane mask) + v_addc
// (cur = 2*cur + bit): 2 VALU per bit, both half-rate with their SGPR operands (38 T
// lane-op/s, profiles/valu_rates_r04.jsonl; a v_sub + v_alignbit form ran at 50.7 T in
// isolation but slower in the kernel, its alignbit chain on `cur` being serial, DESIGN.md
// s9). Each asm block issues all its compares before its adds, so every mask is read >= 2 instructions after it is written (the VALU
// SGPR-write -> carry-read spacing hipcc itself pads with s_nop 1 on gfx950). Loop bits sit
// at compile-time positions (t = 0, 1: 3t..3t+2; t >= 2: 6+4(t-2)..9+4(t-2)) because the
// per-t steps are unrolled by template recursion, so the 32-bit flushes (v_bfrev back to
// the reference's LSB-first order) are static; only the 4 tail bits and the last partial
// word land at n-dependent positions.
//
// `a < av` (float mean, descriptor_transform.hpp:36-39) is evaluated as `a < ceil(sum/n)`:
// for integer a, a < RN(sum/n) <=> a*n < sum (the margin 1/n exceeds half an ulp of any
// value <= 65535) <=> a < ceil(sum/n). ceil(sum/n) = q + (q*n != sum) with
// q = umulhi(sum, magic), magic = ceil(2^32/n): exact because sum < 2^24 makes the
// reciprocal's error < 2^-8 < 1/n (n <= 65).
#define BICOS_CMP(i) "v_cmp_lt_u32_e64 %[m" #i "], %[x" #i "], %[y" #i "]\n\t"
#define BICOS_ADD(i) "v_addc_co_u32_e64 %[c], %[j], %[c], %[c], %[m" #i "]\n\t"
#define BICOS_M(i) [m##i] "=&s"(m##i)
#define BICOS_XY(i) [x##i] "v"(x[i]), [y##i] "v"(y[i])

template <int K>
__device__ __forceinline__ void push_lt(uint32_t& cur, const uint32_t (&x)[4], const uint32_t (&y)[4]) {
    uint64_t m0, m1, m2, m3, j;
    if constexpr (K == 4)
        asm(BICOS_CMP(0) BICOS_CMP(1) BICOS_CMP(2) BICOS_CMP(3) BICOS_ADD(0) BICOS_ADD(1)
                BICOS_ADD(2) BICOS_ADD(3)
            : [c] "+v"(cur), BICOS_M(0), BICOS_M(1), BICOS_M(2), BICOS_M(3), [j] "=&s"(j)
            : BICOS_XY(0), BICOS_XY(1), BICOS_XY(2), BICOS_XY(3));
    else if constexpr (K == 3)
        asm(BICOS_CMP(0) BICOS_CMP(1) BICOS_CMP(2) BICOS_ADD(0) BICOS_ADD(1) BICOS_ADD(2)
            : [c] "+v"(cur), BICOS_M(0), BICOS_M(1), BICOS_M(2), [j] "=&s"(j)
            : BICOS_XY(0), BICOS_XY(1), BICOS_XY(2));
    else if constexpr (K == 2)
        asm(BICOS_CMP(0) BICOS_CMP(1) "s_nop 0\n\t" BICOS_ADD(0) BICOS_ADD(1)
            : [c] "+v"(cur), BICOS_M(0), BICOS_M(1), [j] "=&s"(j)
            : BICOS_XY(0), BICOS_XY(1));
    else if constexpr (K == 1)
        asm(BICOS_CMP(0) "s_nop 1\n\t" BICOS_ADD(0)
            : [c] "+v"(cur), BICOS_M(0), [j] "=&s"(j)
            : BICOS_XY(0));
    (void)m0; (void)m1; (void)m2; (void)m3; (void)j;
}
#undef BICOS_CMP
#undef BICOS_ADD
#undef BICOS_M
#undef BICOS_XY

// Shift the comparisons x[i] < y[i], i < K, into the descriptor at static bit position POS.
template <int POS, int K, int WORDS>
__device__ __forceinline__ void emit_bits(uint32_t& cur, uint32_t (&w)[WORDS], const uint32_t (&x)[4],
                                          const uint32_t (&y)[4]) {
    constexpr int room = 32 - POS % 32;
    if constexpr (K <= room) {
        push_lt<K>(cur, x, y);
        if constexpr (K == room) {
            w[POS / 32] = __builtin_bitreverse32(cur);
            cur = 0;
        }
    } else {
        push_lt<room>(cur, x, y);
        w[POS / 32] = __builtin_bitreverse32(cur);
        cur = 0;
        uint32_t x2[4] = {0, 0, 0, 0}, y2[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = room; i < K; ++i) {
            x2[i - room] = x[i];
            y2[i - room] = y[i];
        }
        push_lt<K - room>(cur, x2, y2);
    }
}

template <int T, int MAXN, int WORDS>
__device__ __forceinline__ void limited_steps(int n, uint32_t thr, const uint32_t (&v)[MAXN],
                                              uint32_t& cur, uint32_t (&w)[WORDS]) {
    if constexpr (T < MAXN - 2) {
        if (T < n - 2) {
            constexpr int pos = T < 2 ? 3 * T : 6 + 4 * (T - 2);
            const uint32_t a = v[T], b = v[T + 1], c = v[T + 2];
            if constexpr (T < 2) {
                const uint32_t x[4] = {a, a, a, 0}, y[4] = {b, c, thr, 0};
                emit_bits<pos, 3, WORDS>(cur, w, x, y);
            } else {
                // ps[t-2] < ps[t]  (descriptor_transform.hpp:52-58; ring slot t % 2)
                const uint32_t x[4] = {a, a, a, v[T - 2] + v[T - 1]}, y[4] = {b, c, thr, a + b};
                emit_bits<pos, 4, WORDS>(cur, w, x, y);
            }
            limited_steps<T + 1, MAXN, WORDS>(n, thr, v, cur, w);
        }
    }
}

// The descriptor of column `col` of the row at element offset `rowoff` (plane pitch `pp`
// elements), n = MAXN when EXACT else n_rt (<= MAXN); magic = ceil(2^32 / n).
template <typename TIn, int WORDS, int MAXN, bool EXACT>
__device__ __forceinline__ void limited_descriptor(const StackReader<TIn>& rd, uint32_t col,
                                                   uint32_t rowoff, uint32_t pp, int n_rt,
                                                   uint32_t magic, uint32_t (&w)[WORDS]) {
    const int n = EXACT ? MAXN : n_rt;

    uint32_t v[MAXN];
#pragma unroll
    for (int t = 0; t < MAXN; ++t)
        if (t < n) v[t] = rd((uint32_t)col, rowoff + (uint32_t)t * pp);
    // the sum from the pair sums ps[t] = v[t] + v[t+1] of even t: the loop below compares
    // those same pair sums (descriptor_transform.hpp:52-58), so they are computed once
    uint32_t sum = 0;
#pragma unroll
    for (int t = 0; t < MAXN; t += 2) {
        if (t + 1 < n)
            sum += v[t] + v[t + 1];
        else if (t < n)
            sum += v[t];
    }
    const uint32_t q = __umulhi(sum, magic);
    const uint32_t thr = q + (q * (uint32_t)n != sum ? 1u : 0u);  // ceil(sum / n)

#pragma unroll
    for (int k = 0; k < WORDS; ++k) w[k] = 0;
    uint32_t cur = 0;
    limited_steps<0, MAXN, WORDS>(n, thr, v, cur, w);

    // bits emitted by the loop, the partial word they leave, then the 4 tail bits
    // (descriptor_transform.hpp:63-68): p[n-2]<p[n-1], p[n-2]<av, p[n-1]<av, ps[n-4]<ps[n-2]
    const int nl = n >= 4 ? 6 + 4 * (n - 4) : 3 * (n - 2);
    const int pw = nl >> 5, pm = nl & 31;
    const uint32_t part = pm ? __builtin_bitreverse32(cur << (32 - pm)) : 0u;
    // the tail samples sit at n-dependent slots: re-load them (cache hits) rather than
    // select them out of the register array
    const uint32_t x = rd((uint32_t)col, rowoff + (uint32_t)(n - 2) * pp);
    const uint32_t y = rd((uint32_t)col, rowoff + (uint32_t)(n - 1) * pp);
    const uint32_t pm2 = n >= 4 ? rd((uint32_t)col, rowoff + (uint32_t)(n - 4) * pp) +
                                      rd((uint32_t)col, rowoff + (uint32_t)(n - 3) * pp)
                                : 0u;
    const uint32_t tail = (uint32_t)(x < y) | ((uint32_t)(x < thr) << 1) | ((uint32_t)(y < thr) << 2) |
                          ((uint32_t)(n < 4 || pm2 < x + y) << 3);
    const int tw = nl >> 5, toff = nl & 31;
#pragma unroll
    for (int k = 0; k < WORDS; ++k) {
        if (k == pw) w[k] |= part;
        if (k == tw) w[k] |= tail << toff;
        if (k == tw + 1 && toff > 28) w[k] |= tail >> (32 - toff);
    }

}

// ---- FULL transform with a compile-time stack size ---------------------------------
//
// descriptor_transform.hpp:75-123: per t < n-2 the bits a<b, a<c, a<av; then the last pair's
// a<b, a<av, b<av; then every pair sum against every pair sum that is not itself or a
// neighbour, ps[t] < ps[i] for t, i < n-1 in (t, i) order -- n^2 - 2n + 3 bits. With n a
// template parameter every bit position is static, so the bits go through the same
// compare -> SGPR mask -> v_addc groups as the LIMITED transform (emit_bits), four at a
// time, with static 32-bit flushes and no per-bit branches.
template <int N>
struct FullOrder {
    static constexpr int M = N >= 3 ? (N - 3) * (N - 2) : 0;  // pair-sum comparisons
    int t[M > 0 ? M : 1], i[M > 0 ? M : 1];
    constexpr FullOrder() : t(), i() {
        int k = 0;
        for (int a = 0; a < N - 1; ++a)
            for (int b = 0; b < N - 1; ++b) {
                if (b == a || b == a - 1 || b == a + 1) continue;
                t[k] = a;
                i[k] = b;
                ++k;
            }
    }
};

// groups of 4 pair-sum comparisons from comparison 4G on, at bit BASE + 4G
template <int N, int WORDS, int BASE, int G>
__device__ __forceinline__ void full_pair_groups(uint32_t& cur, uint32_t (&w)[WORDS],
                                                 const uint32_t (&ps)[N > 1 ? N - 1 : 1]) {
    constexpr FullOrder<N> ord{};
    if constexpr (4 * G < FullOrder<N>::M) {
        constexpr int K = FullOrder<N>::M - 4 * G < 4 ? FullOrder<N>::M - 4 * G : 4;
        uint32_t x[4] = {0, 0, 0, 0}, y[4] = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < K; ++q) {
            x[q] = ps[ord.t[4 * G + q]];
            y[q] = ps[ord.i[4 * G + q]];
        }
        emit_bits<BASE + 4 * G, K, WORDS>(cur, w, x, y);
        full_pair_groups<N, WORDS, BASE, G + 1>(cur, w, ps);
    }
}

template <int T, int N, int WORDS>
__device__ __forceinline__ void full_steps(uint32_t thr, const uint32_t (&v)[N], uint32_t& cur,
                                           uint32_t (&w)[WORDS]) {
    if constexpr (T < N - 2) {
        const uint32_t x[4] = {v[T], v[T], v[T], 0}, y[4] = {v[T + 1], v[T + 2], thr, 0};
        emit_bits<3 * T, 3, WORDS>(cur, w, x, y);
        full_steps<T + 1, N, WORDS>(thr, v, cur, w);
    }
}

template <typename TIn, int WORDS, int N>
__device__ __forceinline__ void full_descriptor(const StackReader<TIn>& rd, uint32_t col,
                                                uint32_t rowoff, uint32_t pp, uint32_t magic,
                                                uint32_t (&w)[WORDS]) {
    static_assert(N >= 2 && N * N - 2 * N + 3 <= 32 * WORDS, "descriptor too narrow");
    uint32_t v[N];
    uint32_t sum = 0;
#pragma unroll
    for (int t = 0; t < N; ++t) {
        v[t] = rd(col, rowoff + (uint32_t)t * pp);
        sum += v[t];
    }
    // a < av  <=>  a < ceil(sum / n) (see limited_descriptor)
    const uint32_t q = __umulhi(sum, magic);
    const uint32_t thr = q + (q * (uint32_t)N != sum ? 1u : 0u);
    uint32_t ps[N > 1 ? N - 1 : 1];
#pragma unroll
    for (int t = 0; t + 1 < N; ++t) ps[t] = v[t] + v[t + 1];
#pragma unroll
    for (int k = 0; k < WORDS; ++k) w[k] = 0;
    uint32_t cur = 0;
    full_steps<0, N, WORDS>(thr, v, cur, w);
    {
        const uint32_t x[4] = {v[N - 2], v[N - 2], v[N - 1], 0}, y[4] = {v[N - 1], thr, thr, 0};
        emit_bits<3 * (N - 2), 3, WORDS>(cur, w, x, y);
    }
    full_pair_groups<N, WORDS, 3 * (N - 2) + 3, 0>(cur, w, ps);
    constexpr int B = N * N - 2 * N + 3;
    if constexpr (B % 32 != 0) w[B / 32] = __builtin_bitreverse32(cur << (32 - B % 32));
}

}  // namespace
}  // namespace bicos_hip
