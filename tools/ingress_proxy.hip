// ingress_proxy.hip -- rank 0's gather ingress of an N-GPU run, rehearsed on one GPU
// (bench.py --root-load proxy). RCCL receives a gather on the root's compute units: a few
// long-lived workgroups (one or two per channel) that copy the peers' data out of their
// receive buffers into the destination while the root's own kernels run. This kernel does
// the same work shape: `nwg` workgroups of 512 threads, each streaming its contiguous slice
// of `bytes` with 8 16-byte loads in flight per thread (the unrolled copy loop RCCL's
// primitives use) -- read + write of the ingress bytes on the root's HBM, on a few CUs, for
// as long as that takes. Test/bench tooling, not product code.
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/ingress_proxy.hip -o build/ingress_proxy.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int THREADS = 512;
constexpr int UNROLL = 8;

__global__ __launch_bounds__(THREADS) void ingress_copy(v4u* __restrict__ dst, const v4u* __restrict__ src,
                                                        size_t n16) {
    const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const size_t b = (size_t)blockIdx.x * per;
    const size_t e = b + per < n16 ? b + per : n16;
    size_t i = b + threadIdx.x;
    for (; i + (UNROLL - 1) * THREADS < e; i += UNROLL * THREADS) {
        v4u v[UNROLL];
#pragma unroll
        for (int k = 0; k < UNROLL; ++k) v[k] = src[i + k * THREADS];
#pragma unroll
        for (int k = 0; k < UNROLL; ++k) dst[i + k * THREADS] = v[k];
    }
    for (; i < e; i += THREADS) dst[i] = src[i];
}

extern "C" int ingress_proxy_launch(void* dst, const void* src, size_t bytes, int nwg, void* stream) {
    if (nwg < 1 || (bytes & 15)) return -1;
    hipLaunchKernelGGL(ingress_copy, dim3(nwg), dim3(THREADS), 0, (hipStream_t)stream, (v4u*)dst,
                       (const v4u*)src, bytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
