// kernels.hpp -- launch interface of the gfx950 BICOS kernels (kernels.hip).
// Plain structs of device pointers and sizes; every launcher is asynchronous on `st`.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace bicos_hip {

struct TransformArgs {
    const void* stack0;     // planar [n][rows][row_pitch] u8/u16
    const void* stack1;     // second stack (or nullptr: transform stack0 only)
    uint32_t* desc0;        // [rows][desc_pitch] uint32
    uint32_t* desc1;
    int n, rows, cols;
    size_t row_pitch;       // elements
    size_t plane_pitch;     // elements
    size_t desc_pitch;      // uint32 words per descriptor row
    uint32_t magic;         // ceil(2^32 / n): exact sum / n by umulhi (set by launch_transform)
    uint32_t stack_bytes;   // bytes addressable from each stack base (< 4 GiB)
};

struct AgreeArgs {
    const int16_t* raw;     // integer disparity from the search
    size_t raw_pitch;
    const void* stack0;
    const void* stack1;
    int n, rows, cols;
    size_t row_pitch, plane_pitch;
    float threshold;
    float step;             // subpixel only
    int nsteps;             // subpixel only: x = -1, -1+step, ... <= 1 (subpixel_steps)
    int has_minvar;
    float minvar;           // already scaled by n (reference cpu.cpp:127)
    void* out;              // dense [rows][cols]
    int out_f32;            // agree: 1 -> float32 output, 0 -> int16 in place semantics
    void* corrmap;          // dense [rows][cols] float (double for DOUBLE) or nullptr
    uint32_t stack_bytes;   // bytes addressable from each stack base (< 4 GiB)
    // Consistency's left-right check inside the agree (launch_agree with fwd != nullptr,
    // aligned stacks): the disparity of pixel (row, col) is consistency_kernel's -- fwd[col]
    // the forward search's best col1 (or -1), rev[col1] the reverse search's best col0 (or
    // -1), both dense [rows][cols] -- instead of raw[col] (reference bicos.hpp:99-106)
    const int16_t* fwd;
    const int16_t* rev;
    int max_lr_diff;
};

struct SearchArgs {
    const uint32_t* desc0;  // the side whose pixels are matched (col0)
    const uint32_t* desc1;  // the side that is searched (col1)
    int16_t* out;
    int rows, cols;
    size_t desc_pitch;      // uint32 words
    size_t out_pitch;       // int16 elements
    int out_mode;           // 0: disparity col0-best (INVALID -32768), 1: best index (-1)
    int chunk;              // set by launch_search
    int tiles_per_row;      // set by launch_search
    int split;              // set by launch_search: waves per col0 group scanning col1 tiles
    int tail_col0;          // set by launch_search_mx: first col0 of the tail workgroups
    int tail_T;             // set by launch_search_mx: their tiles per wave (0: no tail)
    // Compacted col0 (launch_search_mx only; nullptr: every col0 of the row). Row r matches
    // only the distinct col1 >= 0 of keep[r * keep_pitch + c], c < cols, in ascending order,
    // writing out[col]: Consistency's reverse search over the col1 its forward search kept
    // (keep = the forward result, best col1 or -1; reference bicos.hpp:94-101)
    const int16_t* keep;
    size_t keep_pitch;      // int16 elements
    // Consistency's dense-row fast path (launch_search_mx only; nullptr: off). The forward
    // search (out_mode 1, keep == nullptr) writes, per row and 32-col0 tile c0 / 32, how many
    // of its col0 found a valid match (u8, row stride valid_pitch bytes >= ceil(cols / 32)).
    // The compacted reverse search (keep != nullptr) reads its row's counts first: a row
    // whose forward search kept >= 7/8 of its col0 skips the entry prologue and searches
    // every col0 of the row (a superset of the kept col1: the check reads rev only there).
    uint8_t* row_valid;
    size_t valid_pitch;
};

// launch_search_mx_agree: the search and the agree stage (ag.raw unused) that each workgroup
// runs over its own col0 once their search is done. Only those kernel instantiations take
// the agree's arguments (every other search launch keeps the small SearchArgs)
struct SearchAgreeArgs {
    SearchArgs s;
    AgreeArgs ag;
};

struct SearchGeometry {
    int chunk;              // col1 columns per LDS fill
    int waves;              // waves per workgroup
    int R;                  // col0 per lane
    int tiles_per_row;
    int variant;            // 16: packed 16-bit keys (the one VALU search)
    int split;              // packed variant: col1 split across waves of a workgroup (1, 2, 4, 8)
};

struct ConsistencyArgs {
    const int16_t* fwd;     // [rows][cols] best col1 or -1
    const int16_t* rev;     // [rows][cols] best col0 of the reverse search or -1
    int16_t* out;
    int rows, cols;
    size_t out_pitch;
    int max_lr_diff;
};


hipError_t launch_transform(TransformArgs a, int depth, int mode, int words, hipStream_t st);
SearchGeometry search_geometry(int rows, int cols, int words, int max_lds_bytes, int variant = 16,
                               int R = 0, int waves = 0, int split = 0, int cus = 256,
                               int extra_col_bytes = 0);
hipError_t launch_search(SearchArgs a, const SearchGeometry& g, int words, bool nodupes,
                         hipStream_t st);
hipError_t launch_consistency(const ConsistencyArgs& a, hipStream_t st);

// Matrix-core search (search_mx.hip): FP4 MFMA Hamming products, argmin keys in the
// accumulator. Same outputs as launch_search (a.out, a.out_mode).
struct MxGeometry {
    int chunk;              // col1 per LDS fill (multiple of 32)
    int waves;              // waves per workgroup
    int T;                  // 32-col0 tiles per wave (2, 4, 8)
    int tiles_per_row;      // workgroups per row
    int keys;               // 1: one product + xor keys (cols <= 16384), 2: two products
    int ksteps;             // 64-bit K-steps multiplied (<= words / 2; 3 for 256-bit
                            // descriptors with <= 192 used bits)
    int fk;                 // 1: float keys with the column in the free upper half of the
                            // last K-step allowed (<= 64 ksteps - 32 used bits, cols <= 2048;
                            // search_mx.hip KEYS 3, first-minimum searches only)
    // packed Hamming keys (search_mx.hip search_pk_kernel: NoDuplicates, <= 127 used bits,
    // 32/64/128-bit words): used instead of the fields above when pk != 0 and the search
    // is NoDuplicates
    // the row's last workgroup, when it would hold only a few col0: one tail workgroup per
    // row of tail_T (< T) tiles per wave over [tail_col0, cols) (tail_T 0: none)
    int tail_T;
    int tail_col0;
    int pk;
    int pk_T;               // 64-col0 wide tiles per wave (1, 2, 4)
    int pk_chunk;
    int pk_tiles_per_row;
    int pk_tail_col0;       // cols: no tail; else one workgroup per row of 1 wide tile per wave
};
// bits: highest used descriptor bit + 1 when the bits above are known to be zero (0 =
// all of them)
MxGeometry search_mx_geometry(int rows, int cols, int words, int lds_bytes, int T = 0,
                              int waves = 0, int cus = 256, int keys = 0, int bits = 0);
hipError_t launch_search_mx(SearchArgs a, const MxGeometry& g, int words, bool nodupes,
                            hipStream_t st);
// The agree stage fused into the search (one launch): each workgroup, once its waves have
// their col0's results, runs launch_agree's arithmetic over those col0 (a.ag; outputs as
// launch_agree's, a.out still gets the integer map). Only the shapes it is built for: the
// 128-bit NoDuplicates search with 4 or 2 tiles per wave and no tail launch over u8 stacks of n =
// 33, and the packed-key 32-bit search with one wide tile per wave and no tail over u8 stacks
// of n = 8; float, no subpixel step. search_mx_agree_fusable says whether g / the match are one.
bool search_mx_agree_fusable(const MxGeometry& g, int words, bool nodupes, int cols, int n,
                             int depth, bool dbl);
hipError_t launch_search_mx_agree(SearchArgs a, const AgreeArgs& ag, const MxGeometry& g,
                                  hipStream_t st);
// Consistency in one pass (search_mx.hip search_lr_kernel): the forward and the reverse
// search from the same matrix products and the left-right check (reference bicos.hpp:78-113,
// no NoDuplicates), one workgroup per row; a.out gets consistency_kernel's disparity map
// (out_mode 0). Only 256-bit descriptors with 129..154 used bits (`bits`: their count; the
// bits above must be zero) and rows of at most 2048 columns: search_lr_eligible.
bool search_lr_eligible(int words, int bits, int cols);
hipError_t launch_search_lr(SearchArgs a, int words, int bits, int max_lr_diff, hipStream_t st);
hipError_t launch_agree(const AgreeArgs& a, int depth, bool dbl, hipStream_t st);
hipError_t launch_subpixel(const AgreeArgs& a, int depth, bool dbl, hipStream_t st);
// n > 40 (subpixel_wide.hip); launch_subpixel dispatches to it
hipError_t launch_subpixel_wide(const AgreeArgs& a, int depth, bool dbl, hipStream_t st);

}  // namespace bicos_hip
