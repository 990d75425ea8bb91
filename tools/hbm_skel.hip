// hbm_skel.hip -- memory skeletons of the frame's HBM-bound stages (tools/hbm_bound.py):
// the transform's and the agree's exact load/store pattern with the arithmetic stripped, and
// streaming read / read+write kernels over the same byte counts. Timed on inputs that are not
// in the 256 MB last-level cache (the in-frame condition) beside the product kernels, they
// separate "the access pattern's memory bound" from "the kernel's own cost".
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/hbm_skel.hip -o build/libhbm_skel.so
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../libbicos_amd/csrc/stack.hpp"  // the product's buffer-load reader and XCD row map

namespace {
using bicos_hip::StackReader;
using bicos_hip::xcd_rows;

// streaming read of n16 uint4 (4 per thread, coalesced dwordx4); one dword out per workgroup
// only when the xor hits an impossible value, so the loads stay live
__global__ __launch_bounds__(256) void read_x4(const uint4* __restrict__ s, size_t n16,
                                               uint32_t* __restrict__ out) {
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const size_t i = base + (size_t)k * 256;
        if (i < n16) {
            const uint4 v = s[i];
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (x == 0x9E3779B9u) out[blockIdx.x] = x;
}

// read 2 uint4, write 1 (the transform's 207 : 101 MB read : write ratio at cfg2)
__global__ __launch_bounds__(256) void copy_2to1(const uint4* __restrict__ s, uint4* __restrict__ d,
                                                 size_t nout16) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nout16) return;
    const uint4 a = s[2 * i], b = s[2 * i + 1];
    d[i] = make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

// the LIMITED transform's pattern: one pixel per lane, N byte loads (one per plane), four
// descriptor words stored as one uint4 per pixel; grid (cols/256, rows, 2 stacks)
template <int N>
__global__ __launch_bounds__(256) void tf_skel(const uint8_t* __restrict__ s0,
                                               const uint8_t* __restrict__ s1, int cols, size_t pp,
                                               uint32_t bytes, uint4* __restrict__ d0,
                                               uint4* __restrict__ d1) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= cols) return;
    const StackReader<uint8_t> rd(blockIdx.z ? s1 : s0, bytes);
    const uint32_t rowoff = (uint32_t)blockIdx.y * (uint32_t)cols;
    uint32_t v[N];
#pragma unroll
    for (int t = 0; t < N; ++t) v[t] = rd((uint32_t)col, rowoff + (uint32_t)t * (uint32_t)pp);
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < N; ++t) w[t & 3] = (w[t & 3] << 1) ^ v[t];
    (blockIdx.z ? d1 : d0)[(size_t)blockIdx.y * cols + col] = make_uint4(w[0], w[1], w[2], w[3]);
}

// the agree's pattern: the disparity load, the 256-column left tile through LDS by dword
// loads, N right-byte gathers at col - d, disparity + corr stores (8 B per pixel)
template <int N>
__global__ __launch_bounds__(256) void agree_skel(const int16_t* __restrict__ raw,
                                                  const uint8_t* __restrict__ s0,
                                                  const uint8_t* __restrict__ s1, int cols,
                                                  size_t pp, uint32_t bytes, float* __restrict__ out,
                                                  float* __restrict__ corr) {
    __shared__ uint32_t tile[N * 64];
    int t0, row;
    xcd_rows(t0, row);
    const int col0 = t0 * 256, col = col0 + threadIdx.x;
    const bool live = col < cols;
    const uint32_t rowoff = (uint32_t)row * (uint32_t)cols;
    const int d = live ? raw[(size_t)rowoff + col] : -32768;
    const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(s0), (short)0, (int)bytes, 0x00020000);
    const int p0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x / 64);
    const uint32_t lane_b = (uint32_t)col0 + 4u * (threadIdx.x % 64);
    uint32_t w[(N + 3) / 4];
#pragma unroll
    for (int j = 0; j < (N + 3) / 4; ++j) {
        const int p = min(j * 4 + p0, N - 1);
        w[j] = __builtin_amdgcn_raw_buffer_load_b32(r0, lane_b, rowoff + (uint32_t)p * (uint32_t)pp, 0);
    }
    const int c1 = (live && d != -32768 && col - d >= 0 && col - d < cols) ? col - d : 0;
    const StackReader<uint8_t> rd1(s1, bytes);
    uint32_t r[N];
#pragma unroll
    for (int t = 0; t < N; ++t) r[t] = rd1((uint32_t)c1, rowoff + (uint32_t)t * (uint32_t)pp);
#pragma unroll
    for (int j = 0; j < (N + 3) / 4; ++j) {
        const int p = j * 4 + p0;
        if (p < N) tile[p * 64 + threadIdx.x % 64] = w[j];
    }
    __syncthreads();
    if (!live) return;
    const uint8_t* lt = (const uint8_t*)tile + threadIdx.x;
    uint32_t sl = 0, sr = 0;
#pragma unroll
    for (int t = 0; t < N; ++t) {
        sl += lt[t * 256];
        sr += r[t];
    }
    out[(size_t)rowoff + col] = (float)d;
    corr[(size_t)rowoff + col] = (float)(sl ^ sr);
}

}  // namespace

extern "C" {
int skel_read_x4(const void* s, size_t bytes, void* out, hipStream_t st) {
    const size_t n16 = bytes / 16;
    hipLaunchKernelGGL(read_x4, dim3((unsigned)((n16 + 1023) / 1024)), dim3(256), 0, st,
                       (const uint4*)s, n16, (uint32_t*)out);
    return (int)hipGetLastError();
}
int skel_copy_2to1(const void* s, void* d, size_t out_bytes, hipStream_t st) {
    const size_t n = out_bytes / 16;
    hipLaunchKernelGGL(copy_2to1, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const uint4*)s, (uint4*)d, n);
    return (int)hipGetLastError();
}
// n = 33 only (the cfg2 / cfg3 / cfg5 / README stacks); descriptors [rows][cols] uint4
int skel_tf33(const void* s0, const void* s1, int rows, int cols, void* d0, void* d1,
              hipStream_t st) {
    hipLaunchKernelGGL(tf_skel<33>, dim3((cols + 255) / 256, rows, 2), dim3(256), 0, st,
                       (const uint8_t*)s0, (const uint8_t*)s1, cols, (size_t)rows * cols,
                       (uint32_t)((size_t)33 * rows * cols), (uint4*)d0, (uint4*)d1);
    return (int)hipGetLastError();
}
// cols % 256 == 0 (the tile's dword loads are not guarded)
int skel_agree33(const void* raw, const void* s0, const void* s1, int rows, int cols, void* out,
                 void* corr, hipStream_t st) {
    if (cols % 256) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(agree_skel<33>, dim3(cols / 256, rows), dim3(256), 0, st,
                       (const int16_t*)raw, (const uint8_t*)s0, (const uint8_t*)s1, cols,
                       (size_t)rows * cols, (uint32_t)((size_t)33 * rows * cols), (float*)out,
                       (float*)corr);
    return (int)hipGetLastError();
}
}
