// plane_read.hip -- achievable HBM read rate of the agree kernel's access pattern: a
// planar [n][rows][cols] u8 stack, each lane summing one column of n planes (byte loads,
// the agree kernel's form) vs 4 / 16 columns per lane (dword / dwordx4 loads). Decides
// whether the NXC agree kernel (3.2 TB/s at cfg2) is bound by its load-instruction count.
// Build: hipcc --offload-arch=gfx950 -O3 tools/plane_read.hip -o build/plane_read
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int N, int W>  // W = bytes per lane per plane: 1, 4, 16
__global__ __launch_bounds__(256) void rd(const uint8_t* __restrict__ s, uint32_t* out, int rows,
                                         int cols, size_t pp) {
    const int row = blockIdx.y;
    const int c = (blockIdx.x * 256 + threadIdx.x) * W;
    if (c >= cols) return;
    const uint8_t* p = s + (size_t)row * cols + c;
    uint32_t acc = 0;
    if constexpr (W == 1) {
        uint32_t v[N];
#pragma unroll
        for (int t = 0; t < N; ++t) v[t] = p[t * pp];
#pragma unroll
        for (int t = 0; t < N; ++t) acc += v[t] * (t + 1);
    } else if constexpr (W == 4) {
        uint32_t v[N];
#pragma unroll
        for (int t = 0; t < N; ++t) v[t] = *(const uint32_t*)(p + t * pp);
#pragma unroll
        for (int t = 0; t < N; ++t) acc += v[t] * (t + 1);
    } else {
        uint4 v[N];
#pragma unroll
        for (int t = 0; t < N; ++t) v[t] = *(const uint4*)(p + t * pp);
#pragma unroll
        for (int t = 0; t < N; ++t) acc += (v[t].x ^ v[t].y ^ v[t].z ^ v[t].w) * (t + 1);
    }
    out[(size_t)row * cols / W + c / W] = acc;
}

template <int N, int W>
void run(const uint8_t* s, uint32_t* out, int rows, int cols) {
    const size_t pp = (size_t)rows * cols;
    dim3 grid((cols / W + 255) / 256, rows);
    for (int i = 0; i < 30; ++i) hipLaunchKernelGGL((rd<N, W>), grid, dim3(256), 0, 0, s, out, rows, cols, pp);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    const int reps = 50;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((rd<N, W>), grid, dim3(256), 0, 0, s, out, rows, cols, pp);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double bytes = (double)N * pp + (double)rows * cols / W * 4;
    printf("{\"n\": %d, \"bytes_per_lane\": %d, \"us\": %.1f, \"GBps\": %.0f}\n", N, W, ms * 1e3,
           bytes / (ms * 1e-3) / 1e9);
}

int main() {
    const int rows = 1536, cols = 2048;
    uint8_t* s;
    uint32_t* out;
    (void)hipMalloc(&s, (size_t)66 * rows * cols);
    (void)hipMalloc(&out, (size_t)rows * cols * 4);
    (void)hipMemset(s, 7, (size_t)66 * rows * cols);
    run<33, 1>(s, out, rows, cols);
    run<33, 4>(s, out, rows, cols);
    run<33, 16>(s, out, rows, cols);
    run<66, 1>(s, out, rows, cols);
    run<66, 4>(s, out, rows, cols);
    run<66, 16>(s, out, rows, cols);
    return 0;
}
