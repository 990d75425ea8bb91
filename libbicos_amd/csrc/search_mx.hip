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
#include "nxc.hpp"
#include "stack.hpp"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <type_traits>

namespace bicos_hip {

namespace {

constexpr int16_t INVALID_I16 = -32768;

typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr float KEY_BIAS = 256.f;
constexpr float KEY_EPS = 1.f / 32768.f;  // col1 * 2^-15
constexpr float KEY_PAD = 1.0e30f;        // C of columns beyond the image (A = 0 there)

// One-product keys (XK): C = 768 + col1 * 2^-14 keeps every D1 = 768 + x + col1 * 2^-14 in
// the binade [512, 1024) (|x| <= 255), where the ulp is 2^-14: the low 14 mantissa bits of
// D1 ARE col1 and the bits above are x + 256. So bits(D1) ^ 0x3FFF orders by x, then by
// DEScending col1, and its minimum is the last minimum: NoDuplicates costs one v_xor per
// pair instead of a second (negated) product. Needs cols <= 16384.
constexpr float XK_BIAS = 768.f;
constexpr float XK_EPS = 1.f / 16384.f;
constexpr uint32_t XK_COL = 0x3FFFu;
// XK keys are block-relative: C is the same for every block, C = 768 + (XK_K0 + col1 % 32)
// * 2^-14, and the running minima are kept relative to the base col1 B of the block being
// reduced -- their col1 field is col1 - B + XK_K0 (first minimum) and 31 - (col1 - B) (last
// minimum, key ^ 0x3FFF), moved by -32 / +32 per block with ONE integer add each. Both
// fields stay inside [0, 16383] for B <= 16352 (cols <= 16384). This replaces the 16 float
// adds per block that advanced C (which the compiler packed into v_pk_add_f32, expensive
// beside MFMAs) and keeps C in registers that never change.
constexpr int XK_K0 = 16352;
constexpr uint32_t XK_INF = 0x7F000000u;  // "no key yet"; stays huge under the shifts
// KEYS 2 (any block order): the relative col1 fields span +-cols, so C carries a
// mid-range offset instead -- first-minimum field col1 - B + 8160, last-minimum field
// 8223 - (col1 - B) -- which keeps both in [0, 16383] for cols <= 8160.
constexpr int XKF_K0 = 8160;
constexpr int XKF_MAX_COLS = 8160;
// KEYS 3 (float keys, no C matrix): where the descriptors leave the upper lane half of the
// last 64-bit K-step free (e.g. 256-bit words with <= 160 transform bits, cfg4's 154), that
// half carries the column: the right operand holds the binary digits of col1 % 32 there
// (FP4 1, 2, 4, 4+4, 4+4+4+4 in nine elements), the left operand is +1.0 (its descriptor bits
// are 0), and the MFMA scales that half of the right operand by 2^-12. So D = x + (col1 %
// 32) * 2^-12 with C = 0 (an inline constant): 16 VGPRs freer than the XK keys. The running
// minimum is kept relative to the current block base B, D = x + (col1 - B) * 2^-12, moved by
// -32 * 2^-12 per (ascending) block with one float subtract; |col1 - B| < 2048 keeps the
// column term inside (-0.5, 0.5), so floats order by x first and then by col1 (the first
// minimum, v_min3_f32), rint(D) = x, and (D - x) * 4096 = col1 - B exactly (|D| < 256 ->
// ulp 2^-16). NoDuplicates keeps the XK keys (the last minimum needs the bit trick).
constexpr int FK_MAX_COLS = 2048;
constexpr float FK_EPS = 1.f / 4096.f;
constexpr int FK_SCALE_E8M0 = 127 - 12;  // 2^-12

// 32 descriptor bits -> 32 FP4 elements through a byte table: byte q of dword m holds bits
// 8q + 2m (low nibble) and 8q + 2m + 1 (high nibble), i.e. dword m = v_perm of the 4-entry
// table `lut` (one byte per bit pair) selected by the pairs (x >> 2m) & 3 of every byte.
// The order of the bits along K does not matter as long as both operands use the same
// one; 4 v_perm + 7 shift/and per word instead of ~28 shift/or/and.
constexpr uint32_t LUT_A = 0x22200200u;  // right (A): bit 1 -> 1.0 (0x2), 0 -> 0
constexpr uint32_t LUT_B = 0xAAA22A22u;  // left (B): bit 1 -> -1.0 (0xA), 0 -> +1.0 (0x2)
__device__ __forceinline__ v4i expand_bits(uint32_t x, uint32_t lut) {
    v4i r;
#pragma unroll
    for (int m = 0; m < 4; ++m)
        r[m] = (int)__builtin_amdgcn_perm(lut, lut, (x >> (2 * m)) & 0x03030303u);
    return r;
}

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
    return min(min(a, b), c);
}
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) {
    return max(max(a, b), c);
}

__device__ __forceinline__ uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }

constexpr uint32_t KEY_NONE = 0x7F000000u;  // above every key

// min over the 16 keys of a D tile (bits ^ flip) and m; depth-3 tree of v_min3_u32. (The
// keys are positive floats, so v_min3_f32 would do too; measured: it issues at the same half
// rate as v_min3_u32 on gfx950 -- profiles/valu_rates_r02.jsonl -- and the search ran the
// same, cfg2 0.400 vs 0.400 ms, cfg4 0.87 vs 0.86 ms.)
__device__ __forceinline__ uint32_t min16(const v16f& d, uint32_t m, uint32_t flip) {
    // (element copied first: __builtin_bit_cast of a vector-element lvalue reads element 0)
    auto k = [&](int r) { return fbits(d[r]) ^ flip; };
    const uint32_t a0 = umin3(k(0), k(1), k(2)), a1 = umin3(k(3), k(4), k(5));
    const uint32_t a2 = umin3(k(6), k(7), k(8)), a3 = umin3(k(9), k(10), k(11));
    const uint32_t a4 = umin3(k(12), k(13), k(14));
    return umin3(m, umin3(a0, a1, a2), umin3(a3, a4, k(15)));
}
__device__ __forceinline__ uint32_t max16(const v16f& d, uint32_t m) {
    auto k = [&](int r) { return fbits(d[r]); };
    const uint32_t a0 = umax3(k(0), k(1), k(2)), a1 = umax3(k(3), k(4), k(5));
    const uint32_t a2 = umax3(k(6), k(7), k(8)), a3 = umax3(k(9), k(10), k(11));
    const uint32_t a4 = umax3(k(12), k(13), k(14));
    return umax3(m, umax3(a0, a1, a2), umax3(a3, a4, k(15)));
}

// FK column digits of r = col1 % 32 as one lane's 32 FP4 elements (element k = nibble k):
// 1.0 * bit0, 2.0 * bit1, 4.0 * bit2, 4.0 * bit3 (twice), 4.0 * bit4 (four times)
__device__ __forceinline__ v4i fk_digits(int r) {
    uint32_t w0 = 0, w1 = 0;
    w0 |= (r & 1) ? 0x2u : 0u;
    w0 |= (r & 2) ? 0x40u : 0u;
    w0 |= (r & 4) ? 0x600u : 0u;
    w0 |= (r & 8) ? 0x66000u : 0u;
    w0 |= (r & 16) ? 0x66600000u : 0u;
    w1 |= (r & 16) ? 0x6u : 0u;
    return v4i{(int)w0, (int)w1, 0, 0};
}

__device__ __forceinline__ float fmin3(float a, float b, float c) {
    return __builtin_fminf(__builtin_fminf(a, b), c);
}
// min over the 16 float keys of a D tile and m (v_min3_f32 tree)
__device__ __forceinline__ float fmin16(const v16f& d, float m) {
    const float a0 = fmin3(d[0], d[1], d[2]), a1 = fmin3(d[3], d[4], d[5]);
    const float a2 = fmin3(d[6], d[7], d[8]), a3 = fmin3(d[9], d[10], d[11]);
    const float a4 = fmin3(d[12], d[13], d[14]);
    return fmin3(m, fmin3(a0, a1, a2), fmin3(a3, a4, d[15]));
}

__device__ __forceinline__ v16f mfma_fp4(v4i a, v4i b, v16f c) {
    const v8i a8 = {a[0], a[1], a[2], a[3], 0, 0, 0, 0};
    const v8i b8 = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    // cbsz = blgp = 4: both operands FP4 e2m1; zero scales = the unscaled instruction
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 0, 0, 0);
}
// the same with E8M0 scales: sa for this lane's block of the right operand (A), 2^0 for B
__device__ __forceinline__ v16f mfma_fp4_sa(v4i a, v4i b, v16f c, int sa) {
    const v8i a8 = {a[0], a[1], a[2], a[3], 0, 0, 0, 0};
    const v8i b8 = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, sa, 0, 127);
}


// col1 encoded in a key (D1 or D2 bits): key - 256 = +-x + col1 * 2^-15, x integer
__device__ __forceinline__ int key_col(uint32_t key) {
    const float v = bitsf(key) - KEY_BIAS;  // exact
    return (int)((v - floorf(v)) * 32768.f);
}

// KEYS: 0 = float keys (col1 * 2^-15 in C per block; NoDuplicates by a second, negated
//           product), any width;
//       1 = XK keys, blocks in ascending col1 order (cols <= 16384);
//       2 = XK keys in any block order with the last-minimum work skipped where it cannot
//           matter (NoDuplicates, cols <= 8160; see below);
//       3 = FK float keys, column in the free K half, ascending, no NoDuplicates
//           (cols <= 2048, see FK_EPS).
//
// KEYS 2. NoDuplicates needs the LAST column at the minimum cost only to compare it with
// the first; a block none of whose keys reaches the running minimum cost cannot hold it. So
// each tile's block minimum is combined over the two lane halves (tiles in pairs: one
// v_permlane32_swap of two tiles' minima, see pair_reduce) and tested against the tile's
// running first minimum (<= in cost), and the xor + min tree of the last minimum runs only
// for a tile some lane of which passes (one wave-uniform branch per pair). Blocks
// are visited from the wave's own col0 downwards (chunks from the workgroup's, wrapping):
// a stereo match lies at col1 <= col0 within a few blocks, the running minimum reaches it
// early, and the rest of the row skips that half of the VALU work (cfg2 synthetic: ~6 % of
// blocks still do it). The result is exact whatever the data: the order only changes speed.
// Keys stay relative to the base B of the block being reduced (shifts by the signed
// B - B_prev); C = 768 + (8160 + col1 % 32) * 2^-14 keeps both fields in [0, 16383].
//
// A workgroup scans one row for the col0 range [c0_base + tile * waves * T * 32, + waves * T *
// 32), c0_base = a.tail_col0 for the tail launch (launch_mx), else 0.
//
// LIST: the col0 of row r are the distinct col1 >= 0 of row r of a.keep (Consistency's reverse
// search over the col1 its forward search kept, engine.cpp reverse_search), in ascending
// order: entry i is the i-th of them. The workgroup finds its own entries in a prologue
// (list_prologue); the index ranges above run over i, workgroups past the row's count exit,
// and the block order starts REV_AHEAD columns above the wave's highest entry (a reverse
// match lies at col0 = col1 + d, d >= 0 in a rectified pair). The tail split is the full
// search's, in entry space: the main launch takes entries below tail_col0, the tail launch
// the rest (a dense row then costs what it does uncompacted: without the tail, the 4th
// workgroup of a 3300-column row ran 228 entries for a whole-row scan, planted stereo
// NODUPES|CONSISTENCY 2.38 vs 2.24 ms).
// (row, tile) of a compacted (LIST) launch: grid = 8 x ceil(R8 / G) G x tiles_per_row, R8 =
// ceil(rows / 8), G = LIST_GROUP rows. XCD x = bid % 8 owns rows [x R8, (x + 1) R8), and
// within the XCD the order is tile-major per group of G rows: the group's tile 0 workgroups,
// then its tile 1 workgroups, ... Row-major order put the workgroups past a row's count --
// which exit at once -- in a fixed pattern (tiles 2 and 3 of every row at 52 % kept), and the
// dispatcher then ran the live ones on a fixed subset of the CUs: a 52 % list took as long
// as the whole row (random u128, profiles/reverse_search_r05.jsonl). Tile-major over all of
// the XCD's rows fixed that but put a row's workgroups hundreds of workgroups apart, past
// the XCD's L2 (cfg4's reverse search +4.5 %); a group of G = 32 rows x 2 tiles is what an
// XCD holds at once (32 CUs x 2 workgroups), so a row's workgroups run together again.
// Rows past the XCD's range (or past rows) exit.
constexpr int LIST_GROUP = 32;

// LIST prologue scratch at the start of the dynamic LDS (before the first chunk is staged):
// the row's kept-column bitmap (<= 1024 words: cols <= 32767) and 8 wave sums; the
// workgroup's entry columns live after the chunk region
constexpr int LIST_SCRATCH_BYTES = (1024 + 8) * 4;
static_assert(LIST_SCRATCH_BYTES % 16 == 0, "scratch size");

// Consistency's compacted reverse search, the reference's rule (bicos.hpp:94-101,
// bicos.cuh:114,124-131: the reverse search runs only where the forward one found a valid
// match), computed by each workgroup for its own row: the distinct col1 >= 0 of the forward
// result `f` (cols entries) marked in an LDS bitmap, a scan of the words' popcounts, and the
// columns of entries [e0, e0 + ne) written into `ent` by the threads owning their words. Returns the row's entry count (workgroup-uniform). Every
// thread of the workgroup must call it (barriers). Round 5 ran this as a separate kernel
// writing a list to HBM first: 18 us per cfg4 frame; here it overlaps the other resident
// workgroup's matrix-core work.
__device__ int list_prologue(const int16_t* __restrict__ f, int cols, uint32_t* scratch,
                             int16_t* ent, int e0, int ne) {
    const int tid = threadIdx.x, bs = blockDim.x;
    const int nw = (cols + 31) >> 5;
    uint32_t* bits = scratch;
    int* wsum = (int*)(scratch + 1024);
    for (int w = tid; w < nw; w += bs) bits[w] = 0u;
    for (int i = tid; i < ne; i += bs) ent[i] = 0;  // entries past the row's count
    __syncthreads();
    // mark: 8 forward results per thread and 16-byte load where the row is aligned (it is
    // when cols % 8 == 0); a run of results in one bitmap word is one LDS atomic (a stereo
    // row's col1 ascend with col0, so most threads issue one or two)
    auto mark8 = [&](const int (&v)[8]) {
        int cw = -1;
        uint32_t m = 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (v[k] < 0) continue;
            const int w = v[k] >> 5;
            if (w != cw) {
                if (cw >= 0) atomicOr(&bits[cw], m);
                cw = w;
                m = 0u;
            }
            m |= 1u << (v[k] & 31);
        }
        if (cw >= 0) atomicOr(&bits[cw], m);
    };
    if ((reinterpret_cast<uintptr_t>(f) & 15u) == 0) {
        for (int c = 8 * tid; c < cols; c += 8 * bs) {
            int v[8];
            if (c + 8 <= cols) {
                const v4i x = *reinterpret_cast<const v4i*>(f + c);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v[2 * k] = (int)(int16_t)(x[k] & 0xFFFF);
                    v[2 * k + 1] = (int)(int16_t)((uint32_t)x[k] >> 16);
                }
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = c + k < cols ? (int)f[c + k] : -1;
            }
            mark8(v);
        }
    } else {
        for (int c = 8 * tid; c < cols; c += 8 * bs) {
            int v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = c + k < cols ? (int)f[c + k] : -1;
            mark8(v);
        }
    }
    __syncthreads();
    // thread t owns words [t q, t q + q): popcounts, a wave scan and the wave sums give its
    // first entry index; it writes the columns of its set bits that fall in [e0, e0 + ne)
    const int q = (nw + bs - 1) / bs;
    int mine = 0;
    for (int k = 0; k < q; ++k) {
        const int w = tid * q + k;
        mine += w < nw ? __popc(bits[w]) : 0;
    }
    const int lane = tid & 63, wave = tid >> 6, nwaves = bs >> 6;
    int incl = mine;
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
        const int y = __shfl_up(incl, sh);
        if (lane >= sh) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < nwaves; ++w) {
        const int v = wsum[w];
        before += w < wave ? v : 0;
        total += v;
    }
    int e = before + incl - mine;
    if (e < e0 + ne && e + mine > e0) {
        for (int k = 0; k < q; ++k) {
            const int w = tid * q + k;
            uint32_t x = w < nw ? bits[w] : 0u;
            while (x) {
                const int b = __builtin_ctz(x);
                x &= x - 1u;
                if (e >= e0 && e < e0 + ne) ent[e - e0] = (int16_t)(32 * w + b);
                ++e;
            }
        }
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(total);
}

// byte offset of the LIST entry columns in the dynamic LDS: past the chunk region and the
// prologue scratch
__host__ __device__ inline int list_ent_offset(int chunk_bytes) {
    return chunk_bytes > LIST_SCRATCH_BYTES ? (chunk_bytes + 15) / 16 * 16 : LIST_SCRATCH_BYTES;
}
__device__ __forceinline__ void list_row_tile(int tiles_per_row, int rows, int& row, int& tile) {
    const int r8 = (rows + 7) / 8;
    const int j = blockIdx.x / 8;
    const int per_group = LIST_GROUP * tiles_per_row;
    const int g = j / per_group, w = j % per_group;
    tile = w / LIST_GROUP;
    const int r = g * LIST_GROUP + w % LIST_GROUP;  // row within the XCD's range
    row = r < r8 ? (blockIdx.x % 8) * r8 + r : rows;
}
inline int list_grid(int rows, int tiles_per_row) {
    const int r8 = (rows + 7) / 8;
    return 8 * ((r8 + LIST_GROUP - 1) / LIST_GROUP) * LIST_GROUP * tiles_per_row;
}

// Consistency's dense-row fast path (SearchArgs.row_valid): the compacted reverse search's
// workgroup sums its row's per-tile valid counts, written by the forward search's epilogue
// (tile_valid_store), in every wave -- a workgroup-uniform answer without a barrier. A row
// whose forward search kept >= 7/8 of its col0 skips list_prologue (one dependent read of
// the whole forward row, an LDS bitmap and a scan: ~9 us per cfg4 frame, where 98 % of the
// columns are kept) and searches its col0 in order -- every rev the check could read is
// then computed, plus a few it does not read.
__device__ __forceinline__ bool dense_row(const SearchArgs& a, int row) {
    const uint8_t* v = a.row_valid + (size_t)row * a.valid_pitch;
    const int nt = (a.cols + 31) >> 5;
    const int lane = threadIdx.x & 63;
    int sum = 0;
    for (int i = lane; i < nt; i += 64) sum += v[i];
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) sum += __shfl_xor(sum, sh);
    return __builtin_amdgcn_readfirstlane(sum) * 8 >= 7 * a.cols;
}
// forward search epilogue, dense-row fast path: the valid results of one 32-col0 tile (the
// 32 lanes of this lane's half-wave, lane & 31 = col0 % 32) whose col1 `best` lies above the
// previous col0's (a rectified stereo row's matches ascend with col0, so the count stands for
// the DISTINCT col1 the reverse search needs; random descriptors, whose every col0 may be
// valid, count about half), counted into row_valid[row][c0_tile / 32] by the half's writer
__device__ __forceinline__ void tile_valid_store(const SearchArgs& a, int row, int c0_tile,
                                                 bool valid, int best, bool writer) {
    const int v = valid ? best : -1;
    const int prev = __shfl_up(v, 1, 32);  // (the half's first lane: its own value)
    const bool first = (threadIdx.x & 31) == 0;
    const uint64_t bal = __builtin_amdgcn_ballot_w64(valid && (first || v > prev));
    const uint32_t half = (threadIdx.x & 32) ? (uint32_t)(bal >> 32) : (uint32_t)bal;
    if (writer && c0_tile < a.cols)
        a.row_valid[(size_t)row * a.valid_pitch + (c0_tile >> 5)] = (uint8_t)__popc(half);
}

// LIST block order: a wave's blocks start REV_AHEAD columns above its highest entry, a
// workgroup's chunks at the chunk of its highest entry (REV_AHEAD_CHUNK = 0). Starting the
// chunks 64 columns up as well sent every wave through the chunk above first, where only the
// top few entries have their matches: dense rows (planted / low-texture NODUPES|CONSISTENCY
// at 3300 columns) 2.37 / 2.38 ms vs 2.30 / 2.25 (REV_AHEAD 0 / 32: planted 2.35 / 2.32;
// profiles/reverse_search_r05.jsonl)
#ifndef BICOS_REV_AHEAD
#define BICOS_REV_AHEAD 64
#endif
#ifndef BICOS_REV_AHEAD_CHUNK
#define BICOS_REV_AHEAD_CHUNK 0
#endif
constexpr int REV_AHEAD = BICOS_REV_AHEAD;

// The agree stage (kernels.hip agree_reg_kernel, reference agree.hpp:53-93: NXC of the n left
// samples at col and the n right ones at col - d, invalid below the threshold) for the cnt
// col0 from c0 of one row whose integer disparities the workgroup holds in LDS, u8 stacks,
// float, n = N exactly: the search_mx_kernel AG epilogue. Same arithmetic, order and outputs
// as agree_reg_kernel<uint8_t, float, N, true>, so the two are interchangeable bit for bit.
// (Staging the left samples in LDS with dword loads and gathering two pixels' right samples
// per thread before either's arithmetic, as agree_lds_kernel does, measured slower here:
// the fused launch 351 vs 345 us at cfg2, profiles/fused_agree_r05.jsonl.)
template <int N>
__device__ __forceinline__ void fused_agree(const AgreeArgs& g, int row, int c0, int cnt,
                                            const int16_t* raw) {
    const StackReader<uint8_t> rd0(g.stack0, g.stack_bytes), rd1(g.stack1, g.stack_bytes);
    const uint32_t rowoff = (uint32_t)row * (uint32_t)g.row_pitch;
    const uint32_t pp = (uint32_t)g.plane_pitch;
    const int cols = g.cols;
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
        const int col = c0 + i;
        int d = raw[i];
        const int idx1 = col - d;
        const bool inb = d != INVALID_I16 && idx1 >= 0 && idx1 < cols;
        uint32_t l[N], r[N];
        uint32_t sl = 0, sr = 0;
#pragma unroll
        for (int t = 0; t < N; ++t) l[t] = rd0((uint32_t)col, rowoff + (uint32_t)t * pp);
        const uint32_t c1 = inb ? (uint32_t)idx1 : (uint32_t)col;
#pragma unroll
        for (int t = 0; t < N; ++t) r[t] = rd1(c1, rowoff + (uint32_t)t * pp);
#pragma unroll
        for (int t = 0; t < N; ++t) {
            sl += l[t];
            sr += r[t];
        }
        float corr = __builtin_nanf("");
        if (inb) {
            const float m0 = nxc::div_p((float)sl, (float)N);
            const float m1 = nxc::div_p((float)sr, (float)N);
            float cov = 0.f, v0 = 0.f, v1 = 0.f;
#pragma unroll
            for (int t = 0; t < N; ++t) {
                const float x0 = (float)l[t] - m0;
                const float x1 = (float)r[t] - m1;
                cov = nxc::fma_p(x0, x1, cov);
                v0 = nxc::fma_p(x0, x0, v0);
                v1 = nxc::fma_p(x1, x1, v1);
            }
            if (g.has_minvar && (v0 < g.minvar || v1 < g.minvar))
                corr = -1.f;
            else
                corr = nxc::div_p(cov, nxc::sqrt_p(v0 * v1));
            if (corr < g.threshold) d = INVALID_I16;  // NaN passes, as in the reference
        } else {
            d = INVALID_I16;
        }
        const size_t o = (size_t)row * cols + col;
        if (g.out_f32)
            ((float*)g.out)[o] = (float)d;
        else
            ((int16_t*)g.out)[o] = (int16_t)d;
        if (g.corrmap) ((float*)g.corrmap)[o] = corr;
    }
}
constexpr int FUSED_AGREE_N = 33;    // search_mx_kernel AG: 128-bit descriptors (cfg2, cfg5)
constexpr int FUSED_AGREE_N_PK = 8;  // search_pk_kernel AG: 32-bit descriptors (cfg1)
constexpr int REV_AHEAD_CHUNK = BICOS_REV_AHEAD_CHUNK;
// kernel arguments: SearchArgs, plus the agree's for the fused (AG) instantiations only
template <bool AG> struct SearchKArgs { using type = SearchArgs; };
template <> struct SearchKArgs<true> { using type = SearchAgreeArgs; };
__device__ __forceinline__ const SearchArgs& search_part(const SearchArgs& k) { return k; }
__device__ __forceinline__ const SearchArgs& search_part(const SearchAgreeArgs& k) { return k.s; }

template <int WORDS, int KSU, bool NODUPES, int T, int KEYS, bool TAIL, bool LIST, bool AG = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(KSU >= 4 ? 3 : 4)))
void search_mx_kernel(typename SearchKArgs<AG>::type ka) {
    const SearchArgs& a = search_part(ka);
    constexpr bool FK = KEYS == 3;
    static_assert(!FK || !NODUPES, "FK keys: first minimum only");
    constexpr bool XK = KEYS == 1 || KEYS == 2;
    constexpr bool FREE = KEYS == 2;
    static_assert(!FREE || NODUPES, "KEYS 2 is the NoDuplicates search");
    constexpr int K0 = FREE ? XKF_K0 : XK_K0;
    // 64-bit K-steps: KSU <= WORDS / 2 -- the steps past the highest descriptor bit the
    // transform writes are all zero on both sides and contribute nothing (n = 40 LIMITED:
    // 154 of 256 bits -> 3 steps, not 4)
    constexpr int KS = KSU;
    static_assert(KS >= 1 && 2 * KS <= (WORDS >= 2 ? WORDS : 2), "K-steps exceed the descriptor");
    constexpr int WL = 2 * KS;                      // LDS word slots per col1 (W=1: 1 pad)
    extern __shared__ __attribute__((aligned(16))) v4i lds_mx[];  // [WL][chunk]

    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    // XCD-aware order: the tiles of one row on one XCD (shared right row in its L2)
    const int per_xcd = (nwg + 7) / 8;
    int logical = (bid % 8) * per_xcd + bid / 8;
    if (nwg % 8 != 0) logical = bid;
    int row = logical / a.tiles_per_row;
    int tile = logical % a.tiles_per_row;
    if constexpr (LIST) {
        list_row_tile(a.tiles_per_row, a.rows, row, tile);
        if (row >= a.rows) return;
    }
    const int c0_base = TAIL ? a.tail_col0 : 0;

    const int lane = threadIdx.x & 63;
    // wave-uniform, so the block loop's indices and addresses live in SGPRs (the SALU
    // computes them; the VALU issue slots beside the MFMAs are the scarce resource)
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int h = lane >> 5;
    const int j = lane & 31;
    const int cols = a.cols;
    const int chunk = a.chunk;
    const int waves = blockDim.x >> 6;
    const int c0_wave = c0_base + (tile * waves + wave) * (T * 32);
    // col0 entries of this row (LIST: the compacted count, found by the prologue; the
    // workgroup's entry columns in LDS past the chunk region)
    int lcols = cols;
    const int e0 = c0_base + tile * waves * T * 32;
    int16_t* ent = nullptr;
    // LIST, dense row (row_valid): identity entries, no prologue
    bool dense = false;
    if constexpr (LIST) {
        constexpr int WLL = 2 * KSU;
        ent = (int16_t*)((char*)lds_mx + list_ent_offset(WLL * chunk * 16));
        dense = a.row_valid != nullptr && dense_row(a, row);
        if (!dense)
            lcols = list_prologue(a.keep + (size_t)row * a.keep_pitch, cols, (uint32_t*)lds_mx, ent,
                                  e0, waves * T * 32);
        if (!TAIL) lcols = min(lcols, a.tail_col0);  // the tail launch takes the entries past it
        if (e0 >= lcols) return;  // the whole workgroup, past the prologue's barriers
    }
    // LIST: the column of entry i (ascending in i); the block order's start for entries < e
    auto lcol = [&](int i) { return LIST && !dense ? (int)ent[i - e0] : i; };
    auto start_col = [&](int e, int ahead) {
        return LIST ? min(cols - 1, lcol(min(e, lcols) - 1) + ahead) : min(cols - 1, e - 1);
    };

    const uint32_t* __restrict__ row0 = a.desc0 + (size_t)row * a.desc_pitch;
    const uint32_t* __restrict__ row1 = a.desc1 + (size_t)row * a.desc_pitch;

    // B fragments: +1 (0x2) where the left bit is 0, -1 (0xA) where it is 1
    v4i bf[T][KS];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int c0 = c0_wave + 32 * t + j;
        const int cl = c0 < lcols ? lcol(c0) : 0;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int w = 2 * s + h;
            uint32_t x = 0;
            if (c0 < lcols && w < WORDS) x = row0[(size_t)cl * WORDS + w];
            if (WORDS == 8 && KS == 4 && w == 7) x &= 0x7FFFFFFFu;  // bit 255 masked (see below)
            bf[t][s] = expand_bits(x, LUT_B);
        }
    }

    // PAIRS (KEYS 2): the running first minima of tiles 2p / 2p+1 share register mp[p]
    // (lanes 0-31 / 32-63: the halves that write those tiles), see block()
#if defined(BICOS_MX_DIAG) && BICOS_MX_DIAG <= 2
    constexpr bool PAIRS = false;  // diagnostic floors reduce per tile (m1[] must stay live)
#else
    constexpr bool PAIRS = FREE && T % 2 == 0;
#endif
    // one pair per wave: the block loop is software-pipelined (see the FREE chunk loop)
    constexpr bool PIPE = PAIRS && T == 2 && KS <= 3;
    // XK full blocks: the next block's A fragments are read while this one is reduced.
    // Only where the registers allow (paired NoDuplicates tiles, <= 2 K-steps): cfg2 -1.5 %,
    // cfg5 -1 %; with 3 K-steps the extra live fragments spill inside the loop (cfg4 2.3x
    // slower)
    // (FK at 3 K-steps: 25 registers spill even with the C matrix gone)
    constexpr bool PREFETCH = XK && PAIRS && KS <= 2;
    uint32_t m1[T], m2[T], mp[T / 2 > 0 ? T / 2 : 1];
    int b2[T];  // KEYS 2: the base m2[t] is relative to (wave-uniform)
#pragma unroll
    for (int t = 0; t < T; ++t) {
        m1[t] = XK || FK ? XK_INF : KEY_NONE;  // (FK: a huge positive float)
        m2[t] = XK ? XK_INF : 0u;
        b2[t] = 0;
    }
#pragma unroll
    for (int p = 0; p < (T / 2 > 0 ? T / 2 : 1); ++p) mp[p] = XK_INF;

    // row offset of accumulator register r in this lane half
    auto rrow = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };

    v16f d[T], e[T];
    // products of tile `tile` into accumulator slot `slot`
    const int fk_sa = h ? FK_SCALE_E8M0 : 127;  // FK: the column half of the last step x 2^-12
    auto products = [&](int slot, const v4i* af, const v4i* an, const v16f& c1, const v16f& c2,
                        int tile) {
        if constexpr (FK && KS == 1) {
            d[slot] = mfma_fp4_sa(af[0], bf[tile][0], c1, fk_sa);
        } else {
            d[slot] = mfma_fp4(af[0], bf[tile][0], c1);
        }
#pragma unroll
        for (int s = 1; s < KS; ++s) {
            if (FK && s == KS - 1)
                d[slot] = mfma_fp4_sa(af[s], bf[tile][s], d[slot], fk_sa);
            else
                d[slot] = mfma_fp4(af[s], bf[tile][s], d[slot]);
        }
        if constexpr (NODUPES && !XK) {
            e[slot] = mfma_fp4(an[0], bf[tile][0], c2);
#pragma unroll
            for (int s = 1; s < KS; ++s) e[slot] = mfma_fp4(an[s], bf[tile][s], e[slot]);
        }
    };
    // block at base B, the previous one at base bp (XK: the running minima move from bp's
    // frame to B's first)
    auto reduce = [&](int t, int B, int bp) {
#if defined(BICOS_MX_DIAG)  // diagnostic builds only (tools/build_diag.sh): results are wrong
        if constexpr (BICOS_MX_DIAG == 1) {  // MFMA skeleton: one key per tile
            m1[t] = min(m1[t], fbits(d[t][0]));
            return;
        } else if constexpr (BICOS_MX_DIAG == 2) {  // + the first-minimum tree only
            m1[t] = min16(d[t], m1[t], 0u);
            return;
        }
#endif
        if constexpr (FREE) {
            const uint32_t m1s = m1[t] - (uint32_t)(B - bp);
            const uint32_t bm = min16(d[t], KEY_NONE, 0u);      // this half's block minimum
#if defined(BICOS_MX_DIAG) && BICOS_MX_DIAG == 4  // timing only: the last-minimum path never runs
            const bool reach = bm <= (m1s | XK_COL) && bm == 0u;
#else
            const bool reach = bm <= (m1s | XK_COL);           // cost <= running minimum cost
#endif
            const auto sw = __builtin_amdgcn_permlane32_swap(bm, bm, false, false);
            m1[t] = umin3(m1s, sw[0], sw[1]);                  // both halves' minimum
#if defined(BICOS_MX_DIAG) && BICOS_MX_DIAG == 5  // timing only: no last-minimum branch at all
            if (false) {
#else
            if (__builtin_amdgcn_ballot_w64(reach)) {
#endif
                m2[t] = min16(d[t], m2[t] + (uint32_t)(B - b2[t]), XK_COL);
                b2[t] = B;
            }
        } else if constexpr (FK) {
            m1[t] = fbits(fmin16(d[t], bitsf(m1[t]) - 32.f * FK_EPS));
        } else if constexpr (XK) {
            m1[t] = min16(d[t], m1[t] - 32u, 0u);
            if constexpr (NODUPES) m2[t] = min16(d[t], m2[t] + 32u, XK_COL);
        } else {
            m1[t] = min16(d[t], m1[t], 0u);
            if constexpr (NODUPES) m2[t] = max16(e[t], m2[t]);
        }
    };
    int bprev = (XK || FK) && !FREE ? -32 : 0;  // base of the previously reduced block
    // KEYS 2, tiles in pairs (2p, 2p+1) for block base B (accumulators dx, dy): ONE
    // v_permlane32_swap of the two block minima leaves tile 2p's both-halves minimum in
    // lanes 0-31 and tile 2p+1's in lanes 32-63 (swap: vdst lanes 32-63 <-> src lanes 0-31),
    // where the pair's running first minima mp[p] live; one wave-uniform branch per pair,
    // then a scalar test per tile of the ballot's halves. The caller sets bprev = B after.
    auto pair_reduce = [&](int p, int B, const v16f& dx, const v16f& dy) {
        const uint32_t x = min16(dx, KEY_NONE, 0u);
        const uint32_t y = min16(dy, KEY_NONE, 0u);
        const auto sw = __builtin_amdgcn_permlane32_swap(x, y, false, false);
        const uint32_t comb = min((uint32_t)sw[0], (uint32_t)sw[1]);
        const uint32_t ms = mp[p] - (uint32_t)(B - bprev);
#if defined(BICOS_MX_DIAG) && BICOS_MX_DIAG == 4  // timing only: the last-minimum path never runs
        const bool reach = comb <= (ms | XK_COL) && comb == 0u;
#else
        const bool reach = comb <= (ms | XK_COL);  // cost <= running minimum cost
#endif
        mp[p] = min(ms, comb);
#if defined(BICOS_MX_DIAG) && BICOS_MX_DIAG == 5  // timing only: no last-minimum branch at all
        if (reach) m2[2 * p] ^= 0u;
        return;
#endif
        const uint64_t bal = __builtin_amdgcn_ballot_w64(reach);
        // (halves as opaque SGPRs: left alone the compiler tests the upper one with a 64-bit
        // VALU compare)
        uint32_t lo = (uint32_t)bal, hi = (uint32_t)(bal >> 32);
        asm volatile("" : "+s"(lo), "+s"(hi));
        if (lo) {
            m2[2 * p] = min16(dx, m2[2 * p] + (uint32_t)(B - b2[2 * p]), XK_COL);
            b2[2 * p] = B;
        }
        if (hi) {
            m2[2 * p + 1] = min16(dy, m2[2 * p + 1] + (uint32_t)(B - b2[2 * p + 1]), XK_COL);
            b2[2 * p + 1] = B;
        }
    };
    // XK: the C of every block (col1 % 32 only)
    v16f cx;
#pragma unroll
    for (int r = 0; r < 16; ++r) cx[r] = XK_BIAS + (float)(K0 + rrow(r)) * XK_EPS;

    const bool idle = c0_wave >= lcols;  // wave-uniform; still joins the barriers
    const int nchunks = (cols + chunk - 1) / chunk;
    // FREE: chunks downwards from the one holding the workgroup's highest col0
    int cstart = 0;
    if constexpr (FREE) cstart = start_col(c0_base + (tile + 1) * waves * T * 32, REV_AHEAD_CHUNK) / chunk;
    for (int k = 0; k < nchunks; ++k) {
        int ci = FREE ? cstart - k : k;
        if (ci < 0) ci += nchunks;
        const int base = ci * chunk;
        const int ncols = min(chunk, cols - base);
#if defined(BICOS_MX_DIAG) && BICOS_MX_DIAG == 3  // timing only: expand the first chunk only
        const bool expand = k == 0;
#else
        constexpr bool expand = true;
#endif
        if (k && expand) __syncthreads();
        // expand the chunk's right descriptors: one col1 per thread, all its words
        for (int c = threadIdx.x; expand && c < chunk; c += blockDim.x) {
            const int c1 = base + c;
#pragma unroll
            for (int w = 0; w < WL; ++w) {
                uint32_t x = 0;
                if (c1 < cols && w < WORDS) x = row1[(size_t)c1 * WORDS + w];
                if (WORDS == 8 && KS == 4 && w == 7) x &= 0x7FFFFFFFu;
                if (FK && w == WL - 1)  // (the descriptors leave this slot 0: host check)
                    lds_mx[w * chunk + c] = fk_digits(c1 & 31);
                else
                    lds_mx[w * chunk + c] = expand_bits(x, LUT_A);
            }
        }
        if (expand) __syncthreads();
        if (idle) continue;

        const int nfull = ncols / 32;
        const bool partial = (ncols & 31) != 0;
        v16f cc;  // C of the current block: BIAS + col1 * EPS (XK: cx, the same for all)
        if constexpr (FK) {
#pragma unroll
            for (int r = 0; r < 16; ++r) cc[r] = 0.f;  // C = 0: an inline constant
        } else if constexpr (XK) {
            cc = cx;
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) cc[r] = KEY_BIAS + (float)(base + rrow(r)) * KEY_EPS;
        }
        auto block = [&](int b, const v16f& c1, const v16f& c2) {
            const int B = base + 32 * b;
            v4i af[KS], an[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s) af[s] = lds_mx[(2 * s + h) * chunk + 32 * b + j];
#if !defined(BICOS_MX_DIAG) || BICOS_MX_DIAG >= 3
            if constexpr (FREE && PAIRS) {
#pragma unroll
                for (int p = 0; p < T / 2; ++p) {
                    products(0, af, an, c1, c2, 2 * p);
                    products(1, af, an, c1, c2, 2 * p + 1);
                    pair_reduce(p, B, d[0], d[1]);
                }
                bprev = B;
                return;
            }
#endif
            if constexpr (NODUPES && !XK) {
#pragma unroll
                for (int s = 0; s < KS; ++s)
#pragma unroll
                    for (int q = 0; q < 4; ++q) an[s][q] = af[s][q] | (af[s][q] << 2);  // 1.0 -> -1.0
            }
            // tile t+1's products are issued before tile t's keys are reduced, so the MFMAs
            // overlap the reduction (and its branch) within the wave
            products(0, af, an, c1, c2, 0);
#pragma unroll
            for (int t = 0; t < T; ++t) {
                if (t + 1 < T) products(t + 1, af, an, c1, c2, t + 1);
                reduce(t, B, bprev);
            }
            bprev = B;
        };
        // XK full blocks with the A fragments of the next block prefetched: `af` holds block
        // b's fragments on entry; right after the last products that read them are issued,
        // the ds_reads of block `nb` (if >= 0) go out into the same registers, so their
        // latency runs under this block's remaining key reductions
        auto load_af = [&](v4i* af, int b) {
#pragma unroll
            for (int s = 0; s < KS; ++s) af[s] = lds_mx[(2 * s + h) * chunk + 32 * b + j];
        };
        auto block_pf = [&](int b, v4i* af, int nb) {
            const int B = base + 32 * b;
            v4i an[KS];
            if constexpr (FREE && PAIRS) {
#pragma unroll
                for (int p = 0; p < T / 2; ++p) {
                    products(0, af, an, cc, cc, 2 * p);
                    products(1, af, an, cc, cc, 2 * p + 1);
                    if (p + 1 == T / 2 && nb >= 0) load_af(af, nb);
                    pair_reduce(p, B, d[0], d[1]);
                }
            } else {
                products(0, af, an, cc, cc, 0);
                if (T == 1 && nb >= 0) load_af(af, nb);
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    if (t + 1 < T) {
                        products(t + 1, af, an, cc, cc, t + 1);
                        if (t + 2 == T && nb >= 0) load_af(af, nb);
                    }
                    reduce(t, B, bprev);
                }
            }
            bprev = B;
        };
        // the block reaching past the image (last chunk): A = 0 there, so D1 = KEY_PAD,
        // D2 = 0 never win. Ascending orders take it last, FREE first.
        auto partial_block = [&](const v16f& cb) {
            v16f c1, c2;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const bool in = 32 * nfull + rrow(r) < ncols;
                c1[r] = in ? cb[r] : KEY_PAD;
                c2[r] = in ? cb[r] : 0.f;
            }
            block(nfull, c1, c2);
        };
        if constexpr (FREE) {
            if (partial) partial_block(cc);
            // full blocks downwards from the one holding the wave's highest col0 (clamped)
            const int sb = max(0, min(nfull - 1, (start_col(c0_wave + 32 * T, REV_AHEAD) - base) / 32));
#if !defined(BICOS_MX_DIAG) || BICOS_MX_DIAG >= 3
            if constexpr (PIPE) {
                // software pipeline over the blocks (one tile pair per wave): the products of
                // block i+1 are issued before block i is reduced, so the wave's MFMAs stay in
                // flight during its own key reduction (accumulator sets A / B alternate)
                v16f dA[2], dB[2];
                int BA = 0, BB = 0;
                auto issue = [&](int i, v16f* dd) {
                    int b = sb - i;
                    if (b < 0) b += nfull;
                    v4i af[KS];
#pragma unroll
                    for (int s = 0; s < KS; ++s) af[s] = lds_mx[(2 * s + h) * chunk + 32 * b + j];
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        dd[u] = mfma_fp4(af[0], bf[u][0], cc);
#pragma unroll
                        for (int s = 1; s < KS; ++s) dd[u] = mfma_fp4(af[s], bf[u][s], dd[u]);
                    }
                    return base + 32 * b;
                };
                auto finish = [&](int B, const v16f* dd) {
                    pair_reduce(0, B, dd[0], dd[1]);
                    bprev = B;
                };
                if (nfull > 0) {
                    BA = issue(0, dA);
                    for (int i = 0;;) {
                        if (i + 1 < nfull) BB = issue(i + 1, dB);
                        finish(BA, dA);
                        if (++i >= nfull) break;
                        if (i + 1 < nfull) BA = issue(i + 1, dA);
                        finish(BB, dB);
                        if (++i >= nfull) break;
                    }
                }
            } else if constexpr (PREFETCH) {
                auto bidx = [&](int i) {
                    int b = sb - i;
                    return b < 0 ? b + nfull : b;
                };
                v4i af[KS];
                if (nfull > 0) load_af(af, bidx(0));
                for (int i = 0; i < nfull; ++i) block_pf(bidx(i), af, i + 1 < nfull ? bidx(i + 1) : -1);
            } else
#endif
            for (int i = 0; i < nfull; ++i) {
                int b = sb - i;
                if (b < 0) b += nfull;
                block(b, cc, cc);
            }
        } else if constexpr ((XK || FK) && PREFETCH) {
            v4i af[KS];
            if (nfull > 0) load_af(af, 0);
            for (int b = 0; b < nfull; ++b) block_pf(b, af, b + 1 < nfull ? b + 1 : -1);
            if (partial) partial_block(cc);
        } else {
            for (int b = 0; b < nfull; ++b) {
                if constexpr (!XK && !FK) {
                    if (b) {
#pragma unroll
                        for (int r = 0; r < 16; ++r) cc[r] += 32.f * KEY_EPS;  // exact (same binade)
                    }
                }
                block(b, cc, cc);
            }
            if (partial) {
                if constexpr (!XK && !FK) {
                    if (nfull) {
#pragma unroll
                        for (int r = 0; r < 16; ++r) cc[r] += 32.f * KEY_EPS;
                    }
                }
                partial_block(cc);
            }
        }
    }
    if (!AG && idle) return;
    // AG: the workgroup's integer results go through LDS to the fused agree below; the chunk
    // region is reused once every wave is done with its blocks
    int16_t* raw_lds = reinterpret_cast<int16_t*>(lds_mx);
    const int wg_c0 = c0_base + tile * waves * T * 32;
    if constexpr (AG) __syncthreads();

    // the two lane halves hold the even / odd 4-row groups of every block
#pragma unroll
    for (int t = 0; t < T; ++t) {
        if constexpr (FREE) m2[t] += (uint32_t)(bprev - b2[t]);  // into the last block's frame
        if constexpr (PAIRS)  // already merged; valid in the half that writes tile t
            m1[t] = mp[t / 2];
        else if constexpr (FK)
            m1[t] = fbits(__builtin_fminf(bitsf(m1[t]), bitsf((uint32_t)__shfl_xor((int)m1[t], 32))));
        else
            m1[t] = min(m1[t], (uint32_t)__shfl_xor((int)m1[t], 32));
        if constexpr (NODUPES && XK) m2[t] = min(m2[t], (uint32_t)__shfl_xor((int)m2[t], 32));
        else if constexpr (NODUPES) m2[t] = max(m2[t], (uint32_t)__shfl_xor((int)m2[t], 32));
    }
    // best col1 of tile t, and whether it is the only column at the minimum cost
    // (XK: the minima are relative to the base of the last block reduced)
    auto best_of = [&](int t) {
        if constexpr (FK) {
            const float v = bitsf(m1[t]);
            return bprev + (int)((v - __builtin_rintf(v)) * 4096.f);  // exact (see FK_EPS)
        }
        return XK ? (int)(m1[t] & XK_COL) - K0 + bprev : key_col(m1[t]);
    };
    auto unique_of = [&](int t, int best) {
        if constexpr (NODUPES && XK)
            return (int)(XK_COL - K0) - (int)(m2[t] & XK_COL) + bprev == best;
        else if constexpr (NODUPES) return key_col(m2[t]) == best;
        return true;
    };
    int16_t* out = a.out + (size_t)row * a.out_pitch;
    // (lane index made opaque: otherwise the compiler hoists these addresses into the
    // prologue, where they share c0 with the B-fragment loads, and spills them to scratch
    // across the whole search -- 68 MB of scratch writes per cfg2 launch)
    int jo = j;
    asm volatile("" : "+v"(jo));
#pragma unroll
    for (int t = 0; t < T; ++t) {
        if ((t & 1) != h) continue;  // half 0 writes even tiles, half 1 odd tiles
        const int c0i = c0_wave + 32 * t + jo;
        if constexpr (!LIST && !AG) {  // dense-row fast path: this tile's valid count
            if (a.row_valid)
                tile_valid_store(a, row, c0_wave + 32 * t,
                                 c0i < lcols && unique_of(t, best_of(t)), best_of(t), jo == 0);
        }
        if (idle || c0i >= lcols) continue;
        const int c0 = lcol(c0i);
        const int best = best_of(t);
        const bool ok = unique_of(t, best);
        int16_t v;
        if (a.out_mode == 0)
            v = ok ? (int16_t)(c0 - best) : INVALID_I16;
        else
            v = ok ? (int16_t)best : (int16_t)-1;
        // (AG: only the agree reads the integer map, from LDS -- no HBM copy)
        if constexpr (AG)
            raw_lds[c0 - wg_c0] = v;
        else
            out[c0] = v;
    }
    if constexpr (AG) {
        __syncthreads();
        fused_agree<FUSED_AGREE_N>(ka.ag, row, wg_c0, min(waves * T * 32, cols - wg_c0), raw_lds);
    }
}

// ---------------------------------------------------------------------------------------
// Consistency in one pass (round 6): the forward AND the reverse search from the same matrix
// products, then the left-right check, one workgroup per row (reference bicos.hpp:78-113;
// the Consistency variant without NoDuplicates, first minimum both ways).
//
// The forward search reduces each D tile along col1 (16 registers of a lane: 8 v_min3); the
// reverse search needs the same pairs reduced along col0, which the accumulator spreads over
// the 32 lanes of a half-wave. Two launches (forward, then the reverse over the kept col1)
// multiply every pair twice; here the products are shared and the reverse reduction costs a
// lane transposition per block (lr_reduce: 8 v_permlane16_swap + 30 VALU for 32 col1 x the
// wave's 64 col0) instead of a second set of MFMAs.
//
// Keys. The reverse order needs ham itself (|a| varies with col0) and the col0 at the
// minimum; the forward order needs the col1. All three ride in the products, so that
//     D = ham(col0, col1) + (col1 % 32) * 2^-12 + (col0 - c0_wave) * 2^-15
// exactly (ham <= 154, D < 256: 2^-15 is above the ulp):
//  * |a| (popcount of the left descriptor) in the 6 free K elements of the last K-step's
//    lower half (descriptor bits 26..31 of word 2 KS - 2, zero for <= 64 KS - 38 used bits):
//    right (A) constants 1, 6, 6, 6, 6, 6, left (B) FP4 digits with sum = |a| (lr_abs_digits);
//  * col1 % 32 as KEYS 3 (fk_digits in the upper half's A, B = 2.0, the half scaled 2^-13);
//  * col0 - c0_wave = T j + t in 7 more upper-half elements: A constants 0.5, 0.5, 0.5, 0.5, 1,
//    2, 4, B = bit k ? 0.5, 1, 2, 4, 4, 4, 4 : 0 (products 2^-2 .. 2^4, x 2^-13).
// Forward: col0 fixed, so D orders by ham, then col1 (the first minimum); the running minimum
// is kept relative to the block base exactly as KEYS 3. Reverse: col1 fixed, so D orders by
// ham, then col0: the tiles' v_min / v_min3, the lane transposition, + c0_wave * 2^-15, and
// one ds_min_u32 per col1 into the row's LDS array (D >= 0: the bits order like the float).
// Left columns past the image carry |a| digits of 186 > any distance, so they never win.
// col0 of wave w in pass p: c0_wave + T j + t, c0_wave = (p waves + w) * 32 T (interleaved, so
// the col0 offset is the lane and the tile). Passes cover the row; the right row is
// re-expanded per pass (~2 % of the VALU). The epilogue reads fwd[col0] and rev[fwd[col0]]
// from LDS and writes consistency_kernel's disparity (reference bicos.hpp:99-106).
constexpr int LR_MAX_COLS = FK_MAX_COLS;
constexpr int LR_SA_HI = 127 - 13;              // E8M0 2^-13: the upper half of the last step
constexpr float LR_C0_EPS = 1.f / 32768.f;      // col0 * 2^-15
constexpr uint32_t LR_A_W1 = 0x64211110u;       // col0 digit constants, nibbles 1..7 of dword 1
constexpr uint32_t LR_B_W0 = 0x44444444u;       // 2.0 against the col1 digits (dword 0 ...
constexpr uint32_t LR_B_W1 = 0x4u;              // ... and nibble 0 of dword 1)
constexpr uint32_t LR_A_ABS1 = 0x72000000u;     // |a| constants 1, 6 (top byte of dword 1)
constexpr uint32_t LR_A_ABS23 = 0x77000000u;    // 6, 6 (dwords 2 and 3)
constexpr int LR_FREE_BITS = 38;                // 32 upper-half + 6 lower-half K elements
#ifndef BICOS_LR_BL
#define BICOS_LR_BL 1
#endif
constexpr bool LR_BL = BICOS_LR_BL != 0;         // (see search_lr_kernel)

// FP4 code of u / 2 for u in {0, 1, 2, 3, 4, 6, 8, 12}
__device__ __forceinline__ uint32_t lr_code(int u) {
    return u <= 4 ? (uint32_t)u : (u == 6 ? 5u : (u == 8 ? 6u : 7u));
}
// left digits of |a| = n: the top bytes of dwords 1..3 (elements e0..e5, constants 1, 6, ..., 6)
// with n = v0 + 6 (u1 + .. + u5) / 2: v0 = n % 3, q = n / 3 <= 51 as up to four 12s and the
// rest in at most two of {0, 1, 2, 3, 4, 6, 8}. n < 0: the past-the-image column, 186.
__device__ __forceinline__ void lr_abs_digits(int n, uint32_t& b1, uint32_t& b2, uint32_t& b3) {
    if (n < 0) {
        b1 = b2 = b3 = 0x77u;
        return;
    }
    const int v0 = n % 3, q = n / 3;
    const int a = min(4, q / 12), r = q - 12 * a;
    uint32_t cq = 0;  // nibbles of u1..u5
    for (int i = 0; i < a; ++i) cq |= 7u << (4 * i);
    if (a == 4) {
        cq |= lr_code(r) << 16;
    } else {
        const int r1 = r >= 8 ? 8 : (r == 7 ? 6 : (r == 5 ? 4 : r));
        cq |= lr_code(r1) << (4 * a);
        cq |= lr_code(r - r1) << (4 * a + 4);
    }
    b1 = (uint32_t)(2 * v0) | ((cq & 0xFu) << 4);  // v0 in {0, 1, 2}: codes 0, 2, 4
    b2 = (cq >> 4) & 0xFFu;
    b3 = (cq >> 12) & 0xFFu;
}

// The reverse reduction of one block: v[r] = this lane's key for accumulator row r (col1 =
// rrow(r) in its half) and col0 = its lane; returns, per lane, the minimum over the 32 lanes
// of its half of one register's keys (each register's on two adjacent lanes; which register:
// run it on the rows, lr_rows). Steps: rows 0/1 of a half by v_permlane16_swap, then within
// 16-lane rows: lanes 8 apart (row_ror:8), mirrored within 8 (row_half_mirror), 2 apart and 1
// apart (quad_perm), each pairing two registers so that one v_min serves both halves.
template <int CTRL>
__device__ __forceinline__ uint32_t lr_mov(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t lr_reduce(const uint32_t (&v)[16], int lane) {
    uint32_t q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const auto sw = __builtin_amdgcn_permlane16_swap(v[2 * i], v[2 * i + 1], false, false);
        q[i] = min((uint32_t)sw[0], (uint32_t)sw[1]);
    }
    const bool lo8 = (lane & 8) == 0, lo4 = (lane & 4) == 0, lo2 = (lane & 2) == 0;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t u = lo8 ? q[2 * k] : q[2 * k + 1], x = lo8 ? q[2 * k + 1] : q[2 * k];
        w[k] = min(u, lr_mov<0x128>(x));  // row_ror:8
    }
    uint32_t z[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t u = lo4 ? w[2 * k] : w[2 * k + 1], x = lo4 ? w[2 * k + 1] : w[2 * k];
        z[k] = min(u, lr_mov<0x141>(x));  // row_half_mirror
    }
    const uint32_t u = lo2 ? z[0] : z[1], x = lo2 ? z[1] : z[0];
    const uint32_t y = min(u, lr_mov<0x4E>(x));  // quad_perm [2, 3, 0, 1]
    return min(y, lr_mov<0xB1>(y));             // quad_perm [1, 0, 3, 2]
}

template <int WORDS, int KS, int T>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
void search_lr_kernel(SearchArgs a, int max_lr_diff) {
    static_assert(T == 2 || T == 4, "tiles in pairs, <= 128 col0 per wave (7 digit bits)");
    constexpr int WL = 2 * KS;
    static_assert(2 * KS <= WORDS, "K-steps exceed the descriptor");
    extern __shared__ __attribute__((aligned(16))) v4i lds_mx[];  // [WL][chunk] | rev | fwd
    const int row = blockIdx.x;
    if (row >= a.rows) return;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int h = lane >> 5;
    const int j = lane & 31;
    const int cols = a.cols;
    const int chunk = a.chunk;
    const int waves = blockDim.x >> 6;
    const int cols32 = (cols + 31) & ~31;
    uint32_t* rev = reinterpret_cast<uint32_t*>((char*)lds_mx + (size_t)WL * chunk * 16);
    int16_t* fwd = reinterpret_cast<int16_t*>(rev + cols32);
    // LR_BL: the last K-step's B fragments of the wave's tiles live in LDS (one ds_read_b128 per
    // tile and block) -- in registers the 4-tile kernel spilled two of them to scratch, whose
    // reloads per block missed to HBM (PMC: 518 MB read + 129 MB written per cfg4 frame)
    constexpr bool BL = LR_BL && T == 4;
    v4i* bfl = reinterpret_cast<v4i*>(fwd + cols32) + (size_t)wave * T * 64;
    for (int i = threadIdx.x; i < cols32; i += blockDim.x) rev[i] = 0xFFFFFFFFu;

    const uint32_t* __restrict__ row0 = a.desc0 + (size_t)row * a.desc_pitch;
    const uint32_t* __restrict__ row1 = a.desc1 + (size_t)row * a.desc_pitch;
    auto rrow = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };
    // the block-relative col1 whose reverse key lr_reduce leaves in this lane
    int rc1;
    {
        uint32_t v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = (uint32_t)rrow(r);
        rc1 = (int)lr_reduce(v, lane);
    }
    const int sa_hi = h ? LR_SA_HI : 127;
    const int per_pass = waves * T * 32;
    const int passes = (cols + per_pass - 1) / per_pass;
    const int nchunks = (cols + chunk - 1) / chunk;
    for (int pass = 0; pass < passes; ++pass) {
        const int c0_wave = (pass * waves + wave) * (T * 32);
        const bool idle = c0_wave >= cols;  // wave-uniform; still joins the barriers
        // B fragments: +1 (0x2) where the left bit is 0, -1 (0xA) where it is 1, then the
        // digits of |a| (lower half) and the col1 / col0 digit columns (upper half)
        v4i bf[T][KS];
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int c0 = c0_wave + T * j + t;
            const bool in = c0 < cols;
            int pc = 0;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int w = 2 * s + h;
                const uint32_t x = in ? row0[(size_t)c0 * WORDS + w] : 0u;
                pc += __popc(x);
                bf[t][s] = expand_bits(x, LUT_B);
            }
            pc += __shfl_xor(pc, 32);  // both halves' words: |a|
            if (h == 0) {
                uint32_t b1, b2, b3;
                lr_abs_digits(in ? pc : -1, b1, b2, b3);
                v4i& f = bf[t][KS - 1];
                f[1] = (int)(((uint32_t)f[1] & 0x00FFFFFFu) | (b1 << 24));
                f[2] = (int)(((uint32_t)f[2] & 0x00FFFFFFu) | (b2 << 24));
                f[3] = (int)(((uint32_t)f[3] & 0x00FFFFFFu) | (b3 << 24));
            } else {
                const uint32_t c0w = (uint32_t)(T * j + t);
                uint32_t w1 = LR_B_W1;
                constexpr uint32_t code[7] = {0x1u, 0x2u, 0x4u, 0x6u, 0x6u, 0x6u, 0x6u};
#pragma unroll
                for (int k = 0; k < 7; ++k)
                    if (c0w & (1u << k)) w1 |= code[k] << (4 * (k + 1));
                bf[t][KS - 1] = v4i{(int)LR_B_W0, (int)w1, 0, 0};
            }
            if constexpr (BL) bfl[t * 64 + lane] = bf[t][KS - 1];  // (own wave's slots only)
        }
        float m1[T];
#pragma unroll
        for (int t = 0; t < T; ++t) m1[t] = bitsf(XK_INF);
        int bprev = -32;
        const float c0_key = (float)c0_wave * LR_C0_EPS;  // exact

        for (int k = 0; k < nchunks; ++k) {
            const int base = k * chunk;
            const int ncols = min(chunk, cols - base);
            if (k || pass) __syncthreads();
            // expand the chunk's right descriptors, the digit constants in the last step
            for (int c = threadIdx.x; c < chunk; c += blockDim.x) {
                const int c1 = base + c;
#pragma unroll
                for (int w = 0; w < WL; ++w) {
                    v4i v;
                    if (w == WL - 1) {
                        v = fk_digits(c1 & 31);
                        v[1] = (int)((uint32_t)v[1] | LR_A_W1);
                    } else {
                        const uint32_t x = c1 < cols ? row1[(size_t)c1 * WORDS + w] : 0u;
                        v = expand_bits(x, LUT_A);
                        if (w == WL - 2) {
                            v[1] = (int)((uint32_t)v[1] | LR_A_ABS1);
                            v[2] = (int)((uint32_t)v[2] | LR_A_ABS23);
                            v[3] = (int)((uint32_t)v[3] | LR_A_ABS23);
                        }
                    }
                    lds_mx[w * chunk + c] = v;
                }
            }
            __syncthreads();
            if (idle) continue;

            const int nfull = ncols / 32;
            const bool partial = (ncols & 31) != 0;
            // PART: the block reaching past the image (last chunk); its rows past it are set to
            // KEY_PAD after the products (16 v_cndmask per tile in that block only), so every
            // block runs with C = 0 (a C matrix for it made the 4-tile kernel spill)
            auto block = [&](int b, auto part_tag) {
                constexpr bool PART = decltype(part_tag)::value;
                const int B = base + 32 * b;
                v4i af[KS];
                // the A fragments, read again for every tile pair (T = 4: not held across the
                // first pair's key reduction -- 12 registers)
                auto load_af = [&](int p) {
                    int o = 32 * b + j;
                    if (p) asm volatile("" : "+v"(o));  // (a second read, not a copy)
#pragma unroll
                    for (int s = 0; s < KS; ++s) af[s] = lds_mx[(2 * s + h) * chunk + o];
                };
                // (one opaque base per block: read per block -- not hoisted into registers --
                // with the tile in the ds_read's immediate offset)
                int ob = lane;
                if constexpr (BL) asm volatile("" : "+v"(ob));
                auto b_last = [&](int t) {
                    if constexpr (BL)
                        return bfl[ob + t * 64];
                    else
                        return bf[t][KS - 1];
                };
                auto products = [&](int t) {
                    v16f d;
                    if constexpr (KS == 1) {
                        d = mfma_fp4_sa(af[0], b_last(t), v16f{}, sa_hi);
                    } else {
                        d = mfma_fp4(af[0], bf[t][0], v16f{});
#pragma unroll
                        for (int s = 1; s < KS; ++s)
                            d = s == KS - 1 ? mfma_fp4_sa(af[s], b_last(t), d, sa_hi)
                                            : mfma_fp4(af[s], bf[t][s], d);
                    }
                    if constexpr (PART) {
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            if (32 * b + rrow(r) >= ncols) d[r] = KEY_PAD;
                    }
                    return d;
                };
                // tiles in pairs: the forward trees, and the reverse keys' minimum over the
                // tiles (v_min for the first pair, v_min3 after)
                uint32_t v[16];
#pragma unroll
                for (int p = 0; p < T / 2; ++p) {
                    load_af(p);
                    const v16f d0 = products(2 * p), d1 = products(2 * p + 1);
                    m1[2 * p] = fmin16(d0, m1[2 * p] - 32.f * FK_EPS);
                    m1[2 * p + 1] = fmin16(d1, m1[2 * p + 1] - 32.f * FK_EPS);
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        v[r] = p == 0 ? min(fbits(d0[r]), fbits(d1[r]))
                                      : umin3(v[r], fbits(d0[r]), fbits(d1[r]));
                }
                const uint32_t y = fbits(bitsf(lr_reduce(v, lane)) + c0_key);
                if ((lane & 1) == 0) atomicMin(&rev[B + rc1], y);
                bprev = B;
            };
            for (int b = 0; b < nfull; ++b) block(b, std::false_type{});
            if (partial) block(nfull, std::true_type{});
        }
        // this pass's forward results: both lane halves' minima; half h writes the tiles t
        // with t % 2 == h
#pragma unroll
        for (int t = 0; t < T; ++t) {
            m1[t] = __builtin_fminf(m1[t], bitsf((uint32_t)__shfl_xor((int)fbits(m1[t]), 32)));
            const int c0 = c0_wave + T * j + t;
            if ((t & 1) == h && !idle && c0 < cols) {
                const float v = m1[t] - (float)(T * j + t) * LR_C0_EPS;  // exact
                fwd[c0] = (int16_t)(bprev + (int)((v - __builtin_rintf(v)) * 4096.f));
            }
        }
    }
    __syncthreads();
    // the left-right check (bicos.hpp:99-106): rev's key of fwd[col0] holds the reverse
    // search's first col0 at the minimum: bits of D * 2^15 = ham 2^15 + 8 (col1 % 32) + col0
    int16_t* out = a.out + (size_t)row * a.out_pitch;
    for (int c0 = threadIdx.x; c0 < cols; c0 += blockDim.x) {
        const int c1 = fwd[c0];
        const uint32_t kq = (uint32_t)(bitsf(rev[c1]) * 32768.f);  // exact integer
        const int r0 = (int)(kq & 0x7FFFu) - 8 * (c1 & 31);
        const int dlr = c0 - r0;
        out[c0] = (dlr <= max_lr_diff && -dlr <= max_lr_diff) ? (int16_t)((c0 + r0) / 2 - c1)
                                                               : INVALID_I16;
    }
}

// ---------------------------------------------------------------------------------------
// Packed Hamming keys (NoDuplicates, descriptors with <= 127 used bits, 32/64/128-bit words).
//
// The search above spends most of its VALU issue on the first-minimum trees: one v_min3_u32
// per two keys, one key per accumulator register. Here every accumulator register carries
// TWO Hamming distances, and the tree runs on gfx950's v_pk_minimum3_f16 (half rate, four
// keys per instruction; profiles/valu_rates_r03.jsonl), so the reduction per pair halves.
//
// Operands: right A = 1 - 2b in {+1, -1}, left B = -(1 - 2a) / 2 in {-0.5, +0.5} (both exact
// FP4 e2m1), so one K position contributes -(1 - 2a)(1 - 2b) / 2 and K positions sum to
// ham - K / 2 (K = 32 WORDS, the zero bits past the used ones included: they add the same
// -1/2 to every pair). One MFMA multiplies ONE descriptor word: the B lanes of K-half 0 hold
// word w of col0 P, those of K-half 1 word w of col0 Q = P + 32, and the E8M0 scale of the
// K-half-0 lanes is 2^16. With C = 2^23 + 2^16 (K/2) + 0x4B00 + K/2 every D is an integer in
// [2^23, 2^24) (ulp 1), so
//     bits(D) = 0x4B000000 + 2^16 ham(P, col1) + 0x4B00 + ham(Q, col1)
// exactly: the high half is 0x4B00 + ham_P, the low half 0x4B00 + ham_Q, both positive normal
// f16 values whose order is the order of the distances (ham <= 127 keeps each in 7 bits; the
// partial sums of the first words stay inside [0, 127] too). WORDS MFMAs cover 32 col1 x 64
// col0 pairs: the same matrix-core work per pair as the one-product keys.
//
// The keys carry no column. Per wide tile (64 col0) and block (32 col1) the tree gives the
// block's minimum distance per col0 (both lane halves combined by one v_permlane32_swap per
// two tiles, as in pair_reduce); against the running minimum R (packed, per col0):
//   block > R: nothing;  block == R: a second column at the running minimum -> duplicate
//   (tracked as M = min over blocks of (block - R), packed; 0 = tie); block < R: a new
//   minimum: the rare branch finds its first column in the block and whether the block holds
//   it twice ((distance, row) keys through v_perm + v_pk_min_u16, first and reversed rows),
//   and resets M. Any block order gives the same result (a tie with a later-improved minimum
//   is forgotten on the improvement, exactly as the reference's strict '<' scan would).
// Columns beyond the image in the partial block are set to 0x7BFF (the largest finite f16)
// before the tree.
constexpr uint32_t LUT_PA = 0xAAA22A22u;  // right: bit 0 -> +1.0 (0x2), 1 -> -1.0 (0xA)
constexpr uint32_t LUT_PB = 0x11199199u;  // left: bit 0 -> -0.5 (0x9), 1 -> +0.5 (0x1)
constexpr int PK_SCALE_HI = 127 + 16;     // E8M0 2^16 for the K-half-0 (col0 P) lanes
constexpr uint32_t PK_PAD = 0x7BFF7BFFu;
// Lazy drops (round 6). A strict drop of the running minimum used to branch into (distance,
// row) key trees that found its first row and whether the block holds it twice -- one
// wave-uniform branch whenever any of the wave's 128 col0 dropped, ~150 VALU; on random
// descriptors most blocks of a scan take it. Now a drop only records the block base (C) and
// clears the tie marker, and each col0 rescans its final block once after the scan, from the
// right row's raw words staged in LDS: 32 popcounts of WORDS words, the first col1 at the
// minimum and whether it occurs twice (pk_rescan). BICOS_PK_LAZY=0 builds the branch (A/B).
#ifndef BICOS_PK_LAZY
#define BICOS_PK_LAZY 1
#endif
constexpr bool PK_LAZY = BICOS_PK_LAZY != 0;
constexpr int PK_MAX_BITS = 127;
constexpr int PK_MAX_COLS = 32767;

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

// v_pk_minimum3_f16 on two packed positive f16 keys per register
__device__ __forceinline__ uint32_t pkmin3(uint32_t a, uint32_t b, uint32_t c) {
    const h2 x = __builtin_bit_cast(h2, a), y = __builtin_bit_cast(h2, b), z = __builtin_bit_cast(h2, c);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_minimum(__builtin_elementwise_minimum(x, y), z));
}
__device__ __forceinline__ uint32_t pkminu(uint32_t a, uint32_t b) {  // v_pk_min_u16
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pksub(uint32_t a, uint32_t b) {  // v_pk_sub_u16 (wraps)
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) - __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pksign(uint32_t a) {  // 0xFFFF per field with its top bit set
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(i16x2, a) >> (short)15);
}
__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
    return (a & mask) | (b & ~mask);
}

// minimum over the 16 packed keys of a D tile (v_pk_minimum3_f16 tree, 8 instructions)
__device__ __forceinline__ uint32_t pk_tree(const v16f& d) {
    auto k = [&](int r) { return fbits(d[r]); };
    const uint32_t a0 = pkmin3(k(0), k(1), k(2)), a1 = pkmin3(k(3), k(4), k(5));
    const uint32_t a2 = pkmin3(k(6), k(7), k(8)), a3 = pkmin3(k(9), k(10), k(11));
    const uint32_t a4 = pkmin3(k(12), k(13), k(14));
    return pkminu(pkmin3(a0, a1, a2), pkmin3(a3, a4, k(15)));
}
// (distance, row) keys of ONE distance field of a D tile, minimum over this lane half's
// rows: low half distance * 256 + row, high half distance * 256 + (31 - row), row = (r & 3)
// + 8 (r >> 2) (the lane half's 4h is added by the caller) -- the first and the LAST row
// at the minimum distance in one v_pk_min_u16 tree. SEL picks the distance byte of D
// (byte 2: ham_P, byte 0: ham_Q).
template <uint32_t SEL>
__device__ __forceinline__ uint32_t pk_row_keys(const v16f& d) {
    uint32_t k[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t row = (uint32_t)((r & 3) + 8 * (r >> 2));
        // bytes: [row, ham, 31 - row, ham]
        k[r] = __builtin_amdgcn_perm(fbits(d[r]), row | ((31u - row) << 8), SEL);
    }
#pragma unroll
    for (int s = 1; s < 16; s *= 2)
#pragma unroll
        for (int r = 0; r < 16; r += 2 * s) k[r] = pkminu(k[r], k[r + s]);
    return k[0];
}
constexpr uint32_t PK_SEL_P = 0x06010600u;
constexpr uint32_t PK_SEL_Q = 0x04010400u;

__device__ __forceinline__ v16f mfma_pk(v4i a, v4i b, v16f c, int sb) {
    const v8i a8 = {a[0], a[1], a[2], a[3], 0, 0, 0, 0};
    const v8i b8 = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 127, 0, sb);
}

// T wide tiles (64 col0 each) per wave; T = 1 or an even count (tiles reduced in pairs);
// TAIL: the col0 range starts at a.tail_col0 (the tail launch, as search_mx_kernel's);
// LIST: compacted col0 entries (as search_mx_kernel's)
template <int WORDS, int T, bool TAIL, bool LIST, bool AG = false, bool LAZY = PK_LAZY>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
void search_pk_kernel(typename SearchKArgs<AG>::type ka) {
    const SearchArgs& a = search_part(ka);
    static_assert(T == 1 || T % 2 == 0, "wide tiles: 1 or pairs");
    static_assert(!AG || (!TAIL && !LIST), "the fused agree: main launch, every col0");
    static_assert(!AG || WORDS == 1 || WORDS == 4, "the fused agree: cfg1's and cfg2's widths");
    constexpr int NP = T == 1 ? 1 : T / 2;
    extern __shared__ __attribute__((aligned(16))) v4i lds_mx[];  // [WORDS][chunk]

    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int per_xcd = (nwg + 7) / 8;
    int logical = (bid % 8) * per_xcd + bid / 8;
    if (nwg % 8 != 0) logical = bid;
    int row = logical / a.tiles_per_row;
    int tile = logical % a.tiles_per_row;
    if constexpr (LIST) {
        list_row_tile(a.tiles_per_row, a.rows, row, tile);
        if (row >= a.rows) return;
    }

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int h = lane >> 5;
    const int j = lane & 31;
    const int cols = a.cols;
    const int chunk = a.chunk;
    const int waves = blockDim.x >> 6;
    const int c0_base = TAIL ? a.tail_col0 : 0;
    const int c0_wave = c0_base + (tile * waves + wave) * (T * 64);
    int lcols = cols;
    const int e0 = c0_base + tile * waves * T * 64;
    int16_t* ent = nullptr;
    bool dense = false;  // (as search_mx_kernel's)
    if constexpr (LIST) {
        ent = (int16_t*)((char*)lds_mx + list_ent_offset(WORDS * chunk * 16));
        dense = a.row_valid != nullptr && dense_row(a, row);
        if (!dense)
            lcols = list_prologue(a.keep + (size_t)row * a.keep_pitch, cols, (uint32_t*)lds_mx, ent,
                                  e0, waves * T * 64);
        if (!TAIL) lcols = min(lcols, a.tail_col0);  // the tail launch takes the entries past it
        if (e0 >= lcols) return;  // the whole workgroup, past the prologue's barriers
    }
    auto lcol = [&](int i) { return LIST && !dense ? (int)ent[i - e0] : i; };
    auto start_col = [&](int e, int ahead) {
        return LIST ? min(cols - 1, lcol(min(e, lcols) - 1) + ahead) : min(cols - 1, e - 1);
    };

    const uint32_t* __restrict__ row0 = a.desc0 + (size_t)row * a.desc_pitch;
    const uint32_t* __restrict__ row1 = a.desc1 + (size_t)row * a.desc_pitch;

    // B fragments: wide tile t, word w; this lane's col0 is c0_wave + 64 t + lane (K-half h:
    // P = lanes 0-31, Q = lanes 32-63)
    v4i bf[T][WORDS];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int c0 = c0_wave + 64 * t + lane;
        const int cl = c0 < lcols ? lcol(c0) : 0;
#pragma unroll
        for (int w = 0; w < WORDS; ++w) {
            const uint32_t x = c0 < lcols ? row0[(size_t)cl * WORDS + w] : 0u;
            bf[t][w] = expand_bits(x, LUT_PB);
        }
    }
    const int sb = h ? 127 : PK_SCALE_HI;
    constexpr float CBIAS = 8388608.f + 65536.f * (16 * WORDS) + (float)(0x4B00 + 16 * WORDS);
    v16f cb;
#pragma unroll
    for (int r = 0; r < 16; ++r) cb[r] = CBIAS;

    // per pair p (lanes 0-31: tile 2p, lanes 32-63: tile 2p+1; T = 1: all lanes tile 0):
    // running minimum, tie marker, first column of the minimum
    uint32_t R[NP], M[NP], C[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        R[p] = PK_PAD;
        M[p] = 0xFFFFFFFFu;
        C[p] = 0u;
    }
    auto rrow = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };

    // one pair's block minima x (tile 2p) / y (tile 2p+1) at block base B
    auto pair_step = [&](int p, int B, const v16f& dx, const v16f& dy) {
#if defined(BICOS_PK_DIAG) && BICOS_PK_DIAG == 2  // timing only: MFMA skeleton
        M[p] = pkminu(M[p], fbits(dx[0]) ^ fbits(dy[5]));
        return;
#endif
        const uint32_t x = pk_tree(dx);
        const uint32_t y = T == 1 ? x : pk_tree(dy);
        const auto sw = __builtin_amdgcn_permlane32_swap(x, y, false, false);
        const uint32_t comb = pkminu(sw[0], sw[1]);
        const uint32_t diff = pksub(comb, R[p]);
        if constexpr (LAZY) {
            // a strict drop only records the block (branch-free); its first row and whether
            // it holds the minimum twice are found once, after the scan (pk_rescan)
            const uint32_t mi = pksign(diff);
            M[p] = pkminu(M[p], diff) | mi;  // a drop: no tie seen since
            R[p] = bfi(mi, comb, R[p]);
            // (one v_bfi_b32 with the block base as an SGPR operand: left alone, the compiler
            // rebuilt the per-field select from two compares, two cndmasks and a v_perm)
            uint32_t c = C[p];
            asm("v_bfi_b32 %0, %1, %2, %0" : "+v"(c) : "v"(mi), "s"((uint32_t)B * 0x10001u));
            C[p] = c;
            return;
        }
        M[p] = pkminu(M[p], diff);
#if defined(BICOS_PK_DIAG) && BICOS_PK_DIAG == 1  // timing only: the branch never runs
        const bool imp = (diff & 0x80008000u) == 0x80008001u;
#else
        const bool imp = (diff & 0x80008000u) != 0u;
#endif
        if (__builtin_amdgcn_ballot_w64(imp)) {
            // a new running minimum somewhere in the pair: per (tile, distance field) that
            // holds one, the first row at it and whether the block holds it twice
            const uint32_t mi = pksign(diff);
            const uint32_t hoff = h ? 0xFFFC0004u : 0u;  // rows + 4h (low), 31 - rows - 4h (high)
            auto field = [&](auto sel_tag, uint32_t top, int sh) {
                constexpr uint32_t SEL = decltype(sel_tag)::value;
                const uint64_t bal = __builtin_amdgcn_ballot_w64((diff & top) != 0u);
                uint32_t lo = (uint32_t)bal, hi = (uint32_t)(bal >> 32);
                asm volatile("" : "+s"(lo), "+s"(hi));
                if (T == 1) hi = 0;  // (one tile: both halves hold it)
                if (!(lo | hi)) return;
                uint32_t kx = 0, ky = 0;
                if (lo) kx = pk_row_keys<SEL>(dx) + hoff;
                if constexpr (T != 1) {
                    if (hi) ky = pk_row_keys<SEL>(dy) + hoff;
                }
                if (!lo) kx = ky;
                if (!hi) ky = kx;
                const auto sk = __builtin_amdgcn_permlane32_swap(kx, ky, false, false);
                const uint32_t res = pkminu(sk[0], sk[1]);
                const uint32_t first = res & 0x1Fu;
                const uint32_t uniq = first + ((res >> 16) & 0x1Fu) == 31u ? 0xFFFFu : 0u;
                const uint32_t fm = mi & (0xFFFFu << sh);
                R[p] = bfi(fm, comb, R[p]);
                C[p] = bfi(fm, ((uint32_t)B + first) << sh, C[p]);
                M[p] = bfi(fm, uniq << sh, M[p]);
            };
            field(std::integral_constant<uint32_t, PK_SEL_P>{}, 0x80000000u, 16);
            field(std::integral_constant<uint32_t, PK_SEL_Q>{}, 0x00008000u, 0);
        }
    };

    const bool idle = c0_wave >= lcols;  // wave-uniform; still joins the barriers
    const int nchunks = (cols + chunk - 1) / chunk;
    // chunks downwards from the one holding the workgroup's highest col0, blocks downwards
    // from the wave's highest col0 (stereo matches lie at col1 <= col0 within a few blocks,
    // so the running minimum is found early and later blocks rarely take the branch)
    const int cstart = start_col(c0_base + (tile + 1) * waves * T * 64, REV_AHEAD_CHUNK) / chunk;
    for (int k = 0; k < nchunks; ++k) {
        int ci = cstart - k;
        if (ci < 0) ci += nchunks;
        const int base = ci * chunk;
        const int ncols = min(chunk, cols - base);
        if (k) __syncthreads();
        for (int c = threadIdx.x; c < chunk; c += blockDim.x) {
            const int c1 = base + c;
#pragma unroll
            for (int w = 0; w < WORDS; ++w) {
                const uint32_t x = c1 < cols ? row1[(size_t)c1 * WORDS + w] : 0u;
                lds_mx[w * chunk + c] = expand_bits(x, LUT_PA);
            }
        }
        __syncthreads();
        if (idle) continue;

        const int nfull = ncols / 32;
        auto block = [&](int b, bool pad) {
            const int B = base + 32 * b;
#if !defined(BICOS_PK_NOPIN)
            // (C kept in VGPRs: left alone the compiler re-copies it from SGPRs every block)
            asm volatile("" : "+v"(cb));
#endif
            v4i af[WORDS];
#pragma unroll
            for (int w = 0; w < WORDS; ++w) af[w] = lds_mx[w * chunk + 32 * b + j];
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const int tx = T == 1 ? 0 : 2 * p, ty = T == 1 ? 0 : 2 * p + 1;
                v16f dx = mfma_pk(af[0], bf[tx][0], cb, sb);
                v16f dy = dx;
                if constexpr (T != 1) dy = mfma_pk(af[0], bf[ty][0], cb, sb);
#pragma unroll
                for (int w = 1; w < WORDS; ++w) {
                    dx = mfma_pk(af[w], bf[tx][w], dx, sb);
                    if constexpr (T != 1) dy = mfma_pk(af[w], bf[ty][w], dy, sb);
                }
                if (pad) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const bool in = 32 * b + rrow(r) < ncols;
                        dx[r] = in ? dx[r] : bitsf(PK_PAD);
                        dy[r] = in ? dy[r] : bitsf(PK_PAD);
                    }
                }
                pair_step(p, B, dx, dy);
            }
        };
        if ((ncols & 31) != 0) block(nfull, true);
        const int sb0 = max(0, min(nfull - 1, (start_col(c0_wave + 64 * T, REV_AHEAD) - base) / 32));
        for (int i = 0; i < nfull; ++i) {
            int b = sb0 - i;
            if (b < 0) b += nfull;
            block(b, false);
        }
    }
    // AG: the workgroup's integer results go through LDS to the fused agree (as in
    // search_mx_kernel); the chunk region is reused once every wave is done with its blocks.
    // PK_LAZY: the right row's raw words are staged past those results when they fit (one
    // coalesced copy per workgroup, L2-resident), for the rescans below; else read from HBM.
    int16_t* raw_lds = reinterpret_cast<int16_t*>(lds_mx);
    const int wg_c0 = c0_base + tile * waves * T * 64;
    const int row_off = (waves * T * 64 * 2 + 15) & ~15;  // bytes: past raw_lds
    const bool staged = LAZY && (size_t)WORDS * chunk * 16 >= (size_t)row_off + (size_t)cols * WORDS * 4;
    if (!AG && !staged && idle) return;
    if (AG || staged) __syncthreads();
    uint32_t* row_lds = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds_mx) + row_off);
    if (staged) {
        const int nw = cols * WORDS;
        if ((reinterpret_cast<uintptr_t>(row1) & 15u) == 0) {
            for (int i = threadIdx.x; i < nw / 4; i += blockDim.x)
                reinterpret_cast<v4i*>(row_lds)[i] = reinterpret_cast<const v4i*>(row1)[i];
            for (int i = nw / 4 * 4 + threadIdx.x; i < nw; i += blockDim.x) row_lds[i] = row1[i];
        } else {
            for (int i = threadIdx.x; i < nw; i += blockDim.x) row_lds[i] = row1[i];
        }
        __syncthreads();
        if (!AG && idle) return;
    }
    // PK_LAZY: col0 c's final block (base Bb, minimum distance hm) rescanned by popcounts --
    // the first col1 at hm, and whether it occurs twice there; src = the right row's words
    auto rescan = [&](const uint32_t* src, int c, int Bb, uint32_t hm, int& best, bool& uniq) {
        uint32_t aw[WORDS];
#pragma unroll
        for (int w = 0; w < WORDS; ++w) aw[w] = row0[(size_t)c * WORDS + w];
        uint32_t eq = 0;
#pragma unroll 4
        for (int r = 0; r < 32; ++r) {
            const int c1 = Bb + r;
            const int cc = min(c1, cols - 1);  // (past the row: never counted, read in bounds)
            uint32_t hsum = 0;
#pragma unroll
            for (int w = 0; w < WORDS; ++w) hsum = __popc(aw[w] ^ src[(size_t)cc * WORDS + w]) + hsum;
            eq |= (c1 < cols && hsum == hm) ? (1u << r) : 0u;
        }
        best = Bb + (int)__builtin_ctz(eq | 0x80000000u);
        uniq = __popc(eq) == 1;
    };

    int16_t* out = a.out + (size_t)row * a.out_pitch;
    int jo = j;
    asm volatile("" : "+v"(jo));
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        if (T == 1 && h) continue;  // one tile: lanes 0-31 hold it
        const int t = T == 1 ? 0 : 2 * p + h;
#pragma unroll
        for (int f = 0; f < 2; ++f) {  // f = 0: high field (col0 P), 1: low field (Q = P + 32)
            const int c0i = c0_wave + 64 * t + 32 * f + jo;
            const int sh = f ? 0 : 16;
            const bool live = !idle && c0i < lcols;
            int best = (int)((C[p] >> sh) & 0xFFFFu);
            bool ok = ((M[p] >> sh) & 0xFFFFu) != 0u;
            if constexpr (LAZY) {
                // no tie in another block since the drop: count the final block's minima
                if (live && ok) {
                    const uint32_t hm = ((R[p] >> sh) & 0xFFFFu) - 0x4B00u;
                    if (staged)
                        rescan(row_lds, lcol(c0i), best, hm, best, ok);
                    else
                        rescan(row1, lcol(c0i), best, hm, best, ok);
                }
            }
            if constexpr (!LIST && !AG) {  // dense-row fast path: this tile's valid count
                if (a.row_valid)
                    tile_valid_store(a, row, c0_wave + 64 * t + 32 * f, live && ok, best, jo == 0);
            }
            if (!live) continue;
            const int c0 = lcol(c0i);
            int16_t v;
            if (a.out_mode == 0)
                v = ok ? (int16_t)(c0 - best) : INVALID_I16;
            else
                v = ok ? (int16_t)best : (int16_t)-1;
            if constexpr (AG)
                raw_lds[c0 - wg_c0] = v;
            else
                out[c0] = v;
        }
    }
    if constexpr (AG) {
        __syncthreads();
        // (n = 8 with 32-bit descriptors, cfg1; n = 33 with 128-bit, cfg2 / cfg5)
        fused_agree<WORDS == 1 ? FUSED_AGREE_N_PK : FUSED_AGREE_N>(
            ka.ag, row, wg_c0, min(waves * T * 64, cols - wg_c0), raw_lds);
    }
}

// kernel arguments of a launch: the search's, plus the agree's for AG
template <bool AG>
typename SearchKArgs<AG>::type kernel_args(const SearchArgs& a, const AgreeArgs* ag) {
    if constexpr (AG)
        return SearchAgreeArgs{a, *ag};
    else
        return a;
}

// Lazy drops pay a fixed rescan per col0 (~32 popcounts of WORDS words); the drop branch
// pays per drop. Narrow rows (few blocks, few drops on stereo input) keep the branch: cfg1
// (640 columns) 13391 vs 12478-12791 Mpix/s; 3208-3300-column rows take the lazy form: random
// 32-bit NoDuplicates 0.66 vs 1.12-1.14 ms, FULL n = 6 +5 % (FULL n = 8 -1.7 %);
// profiles/pk_lazy_r06.jsonl
constexpr int PK_LAZY_MIN_COLS = 1024;

template <int WORDS, int T, bool TAIL, bool LIST = false, bool AG = false>
hipError_t launch_pk_grid(const SearchArgs& a, int waves, int nwg, hipStream_t st,
                          const AgreeArgs* ag = nullptr) {
    size_t lds = (size_t)WORDS * a.chunk * 16;
    if (LIST) lds = list_ent_offset((int)lds) + (size_t)waves * T * 64 * 2;
    const bool lazy = PK_LAZY && a.cols >= PK_LAZY_MIN_COLS;
    const auto kern = lazy ? search_pk_kernel<WORDS, T, TAIL, LIST, AG, PK_LAZY>
                           : search_pk_kernel<WORDS, T, TAIL, LIST, AG, false>;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void*)kern,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * waves), lds, st, kernel_args<AG>(a, ag));
    return hipGetLastError();
}

// The tail launch's shape: one workgroup per row with only the waves its columns need
// (cols_per_wave each) and a small LDS chunk, so several tail workgroups stay resident per CU
// (the main launch's 64 KiB chunks allow two) -- the tail rows then run in < 2 rounds of
// workgroups instead of 4 (BICOS_TAIL_CHUNK = 0 keeps the main launch's shape; 512 vs 256 vs
// 0: profiles/search_tail_shape_r04.jsonl).
#ifndef BICOS_TAIL_CHUNK
#define BICOS_TAIL_CHUNK 512
#endif
inline void tail_shape(SearchArgs& t, int& waves, int cols_per_wave) {
    t.tiles_per_row = 1;
    if (BICOS_TAIL_CHUNK <= 0) return;
    const int rem = t.cols - t.tail_col0;
    waves = std::max(1, std::min(waves, (rem + cols_per_wave - 1) / cols_per_wave));
    t.chunk = std::min(t.chunk, (int)BICOS_TAIL_CHUNK);
}

// main launch over [0, tail_col0); the tail (one workgroup per row, one wide tile per wave)
// over [tail_col0, cols) when the geometry asked for one (see launch_mx_tt)
// (compacted col0, a.keep: the same split in entry space -- the main workgroups take the
// row's entries below tail_col0, those past the row's count exit; the tail workgroup the
// entries from tail_col0 on, if the row has any)
template <int WORDS, int T>
hipError_t launch_pk(const SearchArgs& a, int waves, hipStream_t st) {
    const bool list = a.keep != nullptr;
    hipError_t e = list ? launch_pk_grid<WORDS, T, false, true>(a, waves, list_grid(a.rows, a.tiles_per_row), st)
                        : launch_pk_grid<WORDS, T, false>(a, waves, a.rows * a.tiles_per_row, st);
    if constexpr (T > 1) {
        if (e == hipSuccess && a.tail_col0 < a.cols) {
            SearchArgs t = a;
            int tw = waves;
            tail_shape(t, tw, 64);
            e = list ? launch_pk_grid<WORDS, 1, true, true>(t, tw, list_grid(a.rows, 1), st)
                     : launch_pk_grid<WORDS, 1, true>(t, tw, a.rows, st);
        }
    }
    return e;
}

template <int WORDS>
hipError_t launch_pk_w(const SearchArgs& a, const MxGeometry& g, hipStream_t st) {
    switch (g.pk_T) {
        case 1: return launch_pk<WORDS, 1>(a, g.waves, st);
        case 2: return launch_pk<WORDS, 2>(a, g.waves, st);
        case 4:
            if constexpr (WORDS <= 2) return launch_pk<WORDS, 4>(a, g.waves, st);
    }
    return hipErrorInvalidValue;
}

template <int WORDS, int KSU, bool NODUPES, int T, int KEYS, bool TAIL, bool LIST = false, bool AG = false>
hipError_t launch_mx_grid(const SearchArgs& a, int waves, int nwg, hipStream_t st,
                          const AgreeArgs* ag = nullptr) {
    constexpr int WL = 2 * KSU;
    size_t lds = (size_t)WL * a.chunk * 16;
    if (LIST) lds = list_ent_offset((int)lds) + (size_t)waves * T * 32 * 2;
    const auto kern = search_mx_kernel<WORDS, KSU, NODUPES, T, KEYS, TAIL, LIST, AG>;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void*)kern,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * waves), lds, st, kernel_args<AG>(a, ag));
    return hipGetLastError();
}

// rows x tiles_per_row workgroups of T tiles per wave over [0, tail_col0); then, when the row's
// last workgroup would hold only a few col0 (tail_col0 < cols), a second launch of one
// workgroup per row with TT < T tiles per wave over [tail_col0, cols). A tail workgroup scans
// the whole row like the others but with fewer tiles, so the remainder no longer costs a full
// T-tile scan: 3208 columns are 3 x 1024 + 136, and the 4th workgroup of every row ran 2 of its
// 8 waves for a full-length scan. (One heterogeneous launch would also fill the main launch's
// last round, but hosting both tile counts in one kernel made the main path spill.)
// Compacted col0 (a.keep) split the same way in entry space (see launch_pk).
template <int WORDS, int KSU, bool NODUPES, int T, int KEYS, int TT>
hipError_t launch_mx_tt(const SearchArgs& a, int waves, hipStream_t st) {
    const bool list = a.keep != nullptr;
    hipError_t e = list ? launch_mx_grid<WORDS, KSU, NODUPES, T, KEYS, false, true>(
                              a, waves, list_grid(a.rows, a.tiles_per_row), st)
                        : launch_mx_grid<WORDS, KSU, NODUPES, T, KEYS, false>(a, waves, a.rows * a.tiles_per_row, st);
    if constexpr (TT == 0) {
        return e;
    } else {
        if (e != hipSuccess) return e;
        SearchArgs t = a;
        int tw = waves;
        tail_shape(t, tw, 32 * TT);
        return list ? launch_mx_grid<WORDS, KSU, NODUPES, TT, KEYS, true, true>(t, tw, list_grid(a.rows, 1), st)
                    : launch_mx_grid<WORDS, KSU, NODUPES, TT, KEYS, true>(t, tw, a.rows, st);
    }
}

template <int WORDS, int KSU, bool NODUPES, int T, int KEYS>
hipError_t launch_mx(const SearchArgs& a, int waves, hipStream_t st) {
    // (tail tiles: 1 or 2, and fewer than the main workgroups'; KEYS 2 only -- the any-order
    // NoDuplicates search, whose block order starts at each wave's own col0)
    if constexpr (KEYS == 2 && T >= 2) {
        if (a.tail_T == 1 && a.tail_col0 < a.cols) return launch_mx_tt<WORDS, KSU, NODUPES, T, KEYS, 1>(a, waves, st);
    }
    if constexpr (KEYS == 2 && T >= 4) {
        if (a.tail_T == 2 && a.tail_col0 < a.cols) return launch_mx_tt<WORDS, KSU, NODUPES, T, KEYS, 2>(a, waves, st);
    }
    // no tail workgroups for these keys / tile counts: the main workgroups cover every col0
    SearchArgs b = a;
    const long per_wg = 32L * waves * T;
    b.tiles_per_row = (int)((a.cols + per_wg - 1) / per_wg);
    b.tail_T = 0;
    b.tail_col0 = a.cols;
    return launch_mx_tt<WORDS, KSU, NODUPES, T, KEYS, 0>(b, waves, st);
}

// Tile counts whose registers fit (checked with -Rpass-analysis=kernel-resource-usage): 8
// tiles only for 32/64-bit descriptors with one key product.
constexpr bool mx_tiles_fit(int words, bool nodupes, int keys, int t) {
    return t <= 4 || (words == 1 && (keys != 0 || !nodupes)) || (words == 2 && !nodupes);
}

template <int WORDS, int KSU, bool NODUPES, int KEYS>
hipError_t launch_mx_k(const SearchArgs& a, const MxGeometry& g, hipStream_t st) {
    if (g.T == 8) {
        if constexpr (mx_tiles_fit(WORDS, NODUPES, KEYS, 8)) {
            return launch_mx<WORDS, KSU, NODUPES, 8, KEYS>(a, g.waves, st);
        } else {  // does not fit: 4 tiles per wave, twice the workgroups per row
            SearchArgs b = a;
            const long per_wg = 32L * g.waves * 4;
            b.tiles_per_row = (int)((a.cols + per_wg - 1) / per_wg);
            b.tail_T = 0;  // (the tail was sized for 8 tiles)
            b.tail_col0 = a.cols;
            return launch_mx<WORDS, KSU, NODUPES, 4, KEYS>(b, g.waves, st);
        }
    }
    switch (g.T) {
        case 2: return launch_mx<WORDS, KSU, NODUPES, 2, KEYS>(a, g.waves, st);
        case 4: return launch_mx<WORDS, KSU, NODUPES, 4, KEYS>(a, g.waves, st);
    }
    return hipErrorInvalidValue;
}

template <int WORDS, int KSU, bool NODUPES>
hipError_t launch_mx_t(const SearchArgs& a, const MxGeometry& g, hipStream_t st) {
    // one-product XK keys by default: with NoDuplicates in any block order up to 8160
    // columns, ascending up to 16384; the two-product float keys beyond that, or when tuned
    // (variant 66)
    if (g.keys == 1) {
        if constexpr (!NODUPES) {
            if (g.fk) return launch_mx_k<WORDS, KSU, NODUPES, 3>(a, g, st);
        }
        if constexpr (NODUPES) {
            if (a.cols <= XKF_MAX_COLS) return launch_mx_k<WORDS, KSU, NODUPES, 2>(a, g, st);
        }
        if (a.cols <= 16384) return launch_mx_k<WORDS, KSU, NODUPES, 1>(a, g, st);
    }
    return launch_mx_k<WORDS, KSU, NODUPES, 0>(a, g, st);
}

template <int WORDS, int KSU>
hipError_t launch_mx_w(const SearchArgs& a, const MxGeometry& g, bool nodupes, hipStream_t st) {
    return nodupes ? launch_mx_t<WORDS, KSU, true>(a, g, st) : launch_mx_t<WORDS, KSU, false>(a, g, st);
}

}  // namespace

MxGeometry search_mx_geometry(int rows, int cols, int words, int lds_bytes, int T, int waves,
                              int cus, int keys, int bits) {
    MxGeometry g;
    g.keys = keys == 2 ? 2 : 1;
    // 64-bit K-steps the products need: all of the descriptor unless the caller knows that
    // the bits past `bits` are zero (transform output); only 256-bit descriptors have a
    // step to drop (129..192 used bits)
    g.ksteps = words >= 2 ? words / 2 : 1;
    if (words == 8 && bits > 0 && bits <= 192) g.ksteps = 3;
    // keys 3 (engine tuned to variant 67): XK keys for the first-minimum searches too (A/B)
    g.fk = keys != 3 && g.keys == 1 && bits > 0 && bits <= 64 * g.ksteps - 32 && cols <= FK_MAX_COLS;
    const int wl = 2 * g.ksteps;
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
        // 4 tiles per wave (2 for 4-step 256-bit descriptors, whose 4-tile B fragments
        // spill: cfg4 1.47 -> 1.09 ms, cfg4f 1.53 -> 0.64 ms; at 3 steps 4 tiles win: cfg4
        // 0.92 -> 0.82 ms; 8 spill for most widths), 2 when the grid would not give every
        // CU about two workgroups (narrow row bands)
        g.T = 2;
        for (int t = g.ksteps >= 4 ? 2 : 4; t >= 2; t /= 2) {
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
    // a short remainder of the row (<= 8 waves x 2 tiles, and at most half of a workgroup)
    // goes to one tail workgroup per row with 1 or 2 tiles per wave (launch_mx_tt), for
    // 4-tile main workgroups: 3208 columns readme 1.127 vs 1.254 ms, FULL n = 12 1.127 vs
    // 1.255; behind 2-tile ones (4-K-step 256-bit, FULL n = 16) it measured slower, 2.15 vs
    // 2.08 ms (profiles/search_tail_r04.jsonl)
    g.tail_T = 0;
    g.tail_col0 = cols;
    const long rem = cols % per_wg;
    if (g.T >= 4 && rem > 0 && cols > per_wg && 2 * rem <= per_wg) {
        const int tt = rem <= 32L * g.waves ? 1 : 2;
        if (tt < g.T && rem <= 32L * g.waves * tt) {
            g.tail_T = tt;
            g.tiles_per_row = (int)(cols / per_wg);
            g.tail_col0 = (int)(cols - rem);
        }
    }
    // packed keys: the default NoDuplicates search for 32/64-bit descriptors (one K-step,
    // where the key reduction, not the matrix products, bounds the one-product search: FULL
    // n = 6 0.63 vs 1.43 ms, n = 8 0.78 vs 0.97 ms at 3208x2200, profiles/search_integ_r04.jsonl),
    // or wherever variant 68 (or BICOS_PK128=1, for 128-bit descriptors with <= 127 used bits)
    // asks for it. With lazy drops (round 6) the 128-bit packed search is faster back to back
    // (cfg2 0.334 vs 0.349 ms, random descriptors 0.382 vs 0.481; profiles/pk128_r06.jsonl), but
    // in the bench's frames it only ties or loses where it matters: cfg2 7889 / 7847 vs 7858 /
    // 7913 Mpix/s, readme -1.2 %, cfg2's 192-row bands of the 8-GPU run -11 % (one wide tile per
    // wave), cfg5 +2.4 % -- so the one-product search stays the 128-bit default.
    // Same workgroup shape, a wide tile = two 32-col0 tiles; the LDS stage holds one expanded
    // word per descriptor word
    // (32/64-bit words need no used-bits hint: a distance is at most 64 <= PK_MAX_BITS)
    static const bool pk128 = [] {
        const char* v = std::getenv("BICOS_PK128");
        return v && !std::strcmp(v, "1");
    }();
    g.pk = (keys == 4 || (keys == 0 && (words <= 2 || (words == 4 && PK_LAZY && pk128)))) &&
           (words <= 2 || (bits > 0 && bits <= PK_MAX_BITS)) && bits <= 32 * words &&
           (words == 1 || words == 2 || words == 4) && cols <= PK_MAX_COLS;
    g.pk_T = g.T >= 2 ? g.T / 2 : 1;
    if (words == 4 && g.pk_T > 2) g.pk_T = 2;  // (4 wide tiles' B fragments do not fit)
    int pchunk = (lds_bytes / (words * 16)) & ~31;
    if (pchunk < 32) pchunk = 32;
    g.pk_chunk = cols32 < pchunk ? cols32 : pchunk;
    const long pk_wg = 64L * g.waves * g.pk_T;
    g.pk_tiles_per_row = (int)((cols + pk_wg - 1) / pk_wg);
    // the packed search's tail: one workgroup per row of one wide tile per wave (FULL n = 6 at
    // 3208 columns: 0.575 vs 0.66 ms, profiles/search_tail_r04.jsonl)
    g.pk_tail_col0 = cols;
    const long pk_rem = cols % pk_wg;
    if (g.pk_T > 1 && pk_rem > 0 && cols > pk_wg && 2 * pk_rem <= pk_wg &&
        pk_rem <= 64L * g.waves) {
        g.pk_tiles_per_row = (int)(cols / pk_wg);
        g.pk_tail_col0 = (int)(cols - pk_rem);
    }
    return g;
}

bool search_mx_agree_fusable(const MxGeometry& g, int words, bool nodupes, int cols, int n,
                             int depth, bool dbl) {
    if (!nodupes || depth != 1 || dbl) return false;
    // packed keys: 32-bit words with one wide tile per wave and n = 8 (cfg1), 128-bit words
    // with one or two and n = 33 (cfg2, cfg5, their row bands); no tail; the raw results (64
    // int16 per wave and wide tile) in the LDS stage (16 B per col1 and word)
    if (g.pk)
        return ((words == 1 && g.pk_T == 1 && n == FUSED_AGREE_N_PK) ||
                (words == 4 && (g.pk_T == 1 || g.pk_T == 2) && n == FUSED_AGREE_N)) &&
               g.pk_tail_col0 == cols && cols <= PK_MAX_COLS &&
               (long)g.pk_chunk * words * 16 >= 128L * g.waves * g.pk_T;
    // launch_mx_t's key choice for this shape is KEYS 2 (NoDuplicates, cols <= XKF_MAX_COLS)
    return words == 4 && g.ksteps == 2 && g.keys == 1 && cols <= XKF_MAX_COLS &&
           (g.T == 4 || g.T == 2) && g.tail_T == 0 && n == FUSED_AGREE_N &&
           g.chunk * 4 * 16 >= 2 * 32 * g.T * g.waves;  // raw in LDS
}

hipError_t launch_search_mx_agree(SearchArgs a, const AgreeArgs& ag, const MxGeometry& g,
                                  hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    if (g.pk) {
        if (a.keep || a.out_mode != 0 || a.cols > PK_MAX_COLS || g.pk_chunk < 32 ||
            (g.pk_chunk & 31) || g.waves < 1 || g.waves > 8 || g.pk_tail_col0 != a.cols)
            return hipErrorInvalidValue;
        a.chunk = g.pk_chunk;
        a.tiles_per_row = g.pk_tiles_per_row;
        a.tail_T = 0;
        a.tail_col0 = a.cols;
        const int nwg = a.rows * a.tiles_per_row;
        if (ag.n == FUSED_AGREE_N_PK && g.pk_T == 1)
            return launch_pk_grid<1, 1, false, false, true>(a, g.waves, nwg, st, &ag);
        if (ag.n == FUSED_AGREE_N && g.pk_T == 1)
            return launch_pk_grid<4, 1, false, false, true>(a, g.waves, nwg, st, &ag);
        if (ag.n == FUSED_AGREE_N && g.pk_T == 2)
            return launch_pk_grid<4, 2, false, false, true>(a, g.waves, nwg, st, &ag);
        return hipErrorInvalidValue;
    }
    if (a.keep || a.out_mode != 0 || a.cols > 32767 || g.chunk < 32 || (g.chunk & 31) ||
        g.waves < 1 || g.waves > 8 || (g.T != 4 && g.T != 2) || g.tail_T != 0)
        return hipErrorInvalidValue;
    a.chunk = g.chunk;
    const long per_wg = 32L * g.waves * g.T;
    a.tiles_per_row = (int)((a.cols + per_wg - 1) / per_wg);
    a.tail_T = 0;
    a.tail_col0 = a.cols;
    // 2 tiles per wave: narrow row bands (N = 8 bands of cfg2, 192 rows)
    if (g.T == 2)
        return launch_mx_grid<4, 2, true, 2, 2, false, false, true>(a, g.waves, a.rows * a.tiles_per_row, st, &ag);
    return launch_mx_grid<4, 2, true, 4, 2, false, false, true>(a, g.waves, a.rows * a.tiles_per_row, st, &ag);
}

// tiles per wave of the one-pass Consistency search (BICOS_LR_T=2: two, A/B)
static int lr_tiles() {
    const char* v = std::getenv("BICOS_LR_T");
    return v && std::atoi(v) == 2 ? 2 : 4;
}

bool search_lr_eligible(int words, int bits, int cols) {
    return words == 8 && bits > 128 && bits <= 3 * 64 - LR_FREE_BITS && cols >= 1 &&
           cols <= LR_MAX_COLS;
}

hipError_t launch_search_lr(SearchArgs a, int words, int bits, int max_lr_diff, hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    if (!search_lr_eligible(words, bits, a.cols) || a.keep || a.out_mode != 0)
        return hipErrorInvalidValue;
    constexpr int KS = 3, WL = 2 * KS;
    // 8 waves of 2 x 32 col0 per pass (fewer for narrow rows); the LDS stage as the KEYS 3
    // search's (64 KiB) plus the row's reverse keys and forward results
    const int T = lr_tiles();
    const int waves = std::min(8, (a.cols + 32 * T - 1) / (32 * T));
    const int cols32 = (a.cols + 31) & ~31;
    // two workgroups per CU: <= 80 KiB each for the stage, the row's keys and results and (4
    // tiles) the B fragments of the last K-step; cfg4: 384-column chunks
    const size_t fixed = (size_t)cols32 * 6 + (LR_BL && T == 4 ? (size_t)waves * T * 64 * 16 : 0);
    int chunk = (int)((80 * 1024 - fixed) / (WL * 16)) & ~31;
    if (chunk > cols32) chunk = cols32;
    if (chunk < 32) return hipErrorInvalidValue;
    a.chunk = chunk;
    const size_t lds = (size_t)WL * chunk * 16 + fixed;
    const auto kern = T == 4 ? search_lr_kernel<8, KS, 4> : search_lr_kernel<8, KS, 2>;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void*)kern,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(a.rows), dim3(64 * waves), lds, st, a, max_lr_diff);
    return hipGetLastError();
}

hipError_t launch_search_mx(SearchArgs a, const MxGeometry& g, int words, bool nodupes,
                            hipStream_t st) {
    if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
    if (a.cols > 32767 || g.chunk < 32 || (g.chunk & 31) || g.waves < 1 || g.waves > 8)
        return hipErrorInvalidValue;
    if (g.pk && nodupes) {
        if (a.cols > PK_MAX_COLS || g.pk_chunk < 32 || (g.pk_chunk & 31)) return hipErrorInvalidValue;
        a.chunk = g.pk_chunk;
        a.tiles_per_row = g.pk_tiles_per_row;
        a.tail_T = 0;
        a.tail_col0 = g.pk_tail_col0;
        switch (words) {
            case 1: return launch_pk_w<1>(a, g, st);
            case 2: return launch_pk_w<2>(a, g, st);
            case 4: return launch_pk_w<4>(a, g, st);
        }
        return hipErrorInvalidValue;
    }
    a.chunk = g.chunk;
    a.tiles_per_row = g.tiles_per_row;
    a.tail_T = g.tail_T;
    a.tail_col0 = g.tail_col0;
    switch (words) {
        case 1: return launch_mx_w<1, 1>(a, g, nodupes, st);
        case 2: return launch_mx_w<2, 1>(a, g, nodupes, st);
        case 4: return launch_mx_w<4, 2>(a, g, nodupes, st);
        case 8:
            if (g.ksteps == 3) return launch_mx_w<8, 3>(a, g, nodupes, st);
            return launch_mx_w<8, 4>(a, g, nodupes, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace bicos_hip
