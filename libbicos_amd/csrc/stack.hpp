// stack.hpp -- device helpers shared by the kernels that read the image stacks
// (transform and agree in kernels.hip, the subpixel refine in subpixel.hpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bicos_hip {
namespace {

// Raw buffer loads of an image stack: 128-bit resource built from uniform values, uniform
// (SGPR) byte offset of the plane/row, 32-bit per-lane byte offset -- no VALU address math
// per load (guide T8). Stacks are limited to < 4 GiB (checked by the engine).
template <typename TIn>
struct StackReader {
    __amdgpu_buffer_rsrc_t r;
    __device__ __forceinline__ StackReader(const void* base, uint32_t bytes)
        : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                               0x00020000)) {}
    __device__ __forceinline__ uint32_t operator()(uint32_t lane_elem, uint32_t uniform_elem) const {
        if constexpr (sizeof(TIn) == 1)
            return __builtin_amdgcn_raw_buffer_load_b8(r, lane_elem, uniform_elem, 0);
        else
            return __builtin_amdgcn_raw_buffer_load_b16(r, lane_elem * 2u, uniform_elem * 2u, 0);
    }
};

// (column tile, row) of a (tiles x rows) grid, remapped so that each XCD gets a run of
// whole rows: workgroups are dispatched round-robin over the 8 XCDs in linear order, so
// without this neighbouring column tiles land on different XCDs and the right-image
// windows they share (col - d, col1 +- 1) are fetched into two L2s.
__device__ __forceinline__ void xcd_rows(int& tile, int& row) {
    const int gx = gridDim.x;
    const int nwg = gx * gridDim.y;
    if (nwg % 8) {
        tile = blockIdx.x;
        row = blockIdx.y;
        return;
    }
    const int bid = blockIdx.y * gx + blockIdx.x;
    const int logical = (bid % 8) * (nwg / 8) + bid / 8;
    tile = logical % gx;
    row = logical / gx;
}

}  // namespace
}  // namespace bicos_hip
