// mfma_rate.hip -- sustained rate of the FP4 block-scaled MFMA on this MI355X:
// v_mfma_scale_f32_32x32x64_f8f6f4 and _16x16x128_ with FP4 (e2m1) operands of random
// bits, CHAINS independent accumulators per wave (1 = back-to-back dependent), WAVES waves
// per SIMD. Prints TFLOP/s and cycles per MFMA at the nominal 2.4 GHz. The search kernel's
// MFMA skeleton (tools/build_diag.sh) is judged against these numbers.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o build/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int CHAINS, bool SC = false>
__global__ __launch_bounds__(256) void k32(const int* seed, float* out, int iters) {
    // SC: per-lane E8M0 scales from registers (the packed-key search's 2^16 / 2^0 on B)
    const int sa = 127 + (seed[0] & 0), sb = (threadIdx.x & 32) ? 127 : 143 + (seed[1] & 0);
    const int l = threadIdx.x;
    v8i a, b;
    for (int q = 0; q < 8; ++q) {
        a[q] = q < 4 ? seed[(l * 7 + q) & 255] : 0;
        b[q] = q < 4 ? seed[(l * 11 + q + 3) & 255] : 0;
    }
    v16f acc[CHAINS];
    for (int c = 0; c < CHAINS; ++c)
        for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < CHAINS; ++c)
            acc[c] = SC ? __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[c], 4, 4, 0, sa, 0, sb)
                        : __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[c], 4, 4, 0, 0, 0, 0);
    float s = 0.f;
    for (int c = 0; c < CHAINS; ++c)
        for (int r = 0; r < 16; ++r) s += acc[c][r];
    out[blockIdx.x * blockDim.x + l] = s;
}

template <int CHAINS>
__global__ __launch_bounds__(256) void k16(const int* seed, float* out, int iters) {
    const int l = threadIdx.x;
    v8i a, b;
    for (int q = 0; q < 8; ++q) {
        a[q] = q < 4 ? seed[(l * 7 + q) & 255] : 0;
        b[q] = q < 4 ? seed[(l * 11 + q + 3) & 255] : 0;
    }
    v4f acc[CHAINS];
    for (int c = 0; c < CHAINS; ++c)
        for (int r = 0; r < 4; ++r) acc[c][r] = 0.f;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < CHAINS; ++c)
            acc[c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[c], 4, 4, 0, 0, 0, 0);
    float s = 0.f;
    for (int c = 0; c < CHAINS; ++c)
        for (int r = 0; r < 4; ++r) s += acc[c][r];
    out[blockIdx.x * blockDim.x + l] = s;
}

template <typename K>
void run(const char* name, K kern, double flop_per_mfma, int chains, int waves_per_simd,
         const int* seed, float* out) {
    const int iters = 4000;
    // 256 threads = 4 waves per workgroup; waves_per_simd workgroups per CU
    const int grid = 256 * waves_per_simd;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, seed, out, iters);  // warm + clocks
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, seed, out, iters);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, seed, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double mfmas = (double)grid * 4 * iters * chains * reps;  // per wave
    const double tflops = mfmas * flop_per_mfma / (ms * 1e-3) / 1e12;
    const double per_simd = mfmas / 1024.0;
    printf("{\"mfma\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"TFLOPs\": %.0f, "
           "\"cycles_per_mfma_at_2.4GHz\": %.1f}\n",
           name, chains, waves_per_simd, tflops, ms * 1e-3 * 2.4e9 / per_simd);
}

int main() {
    int* seed;
    float* out;
    hipMalloc(&seed, 256 * 4);
    hipMalloc(&out, 256 * 8 * 256 * 4);
    int h[256];
    unsigned x = 0x12345678u;
    for (int i = 0; i < 256; ++i) {
        x = x * 1664525u + 1013904223u;
        h[i] = (int)(x & 0x3B3B3B3Bu);  // e2m1 nibbles of magnitude <= 1.5: no overflow
    }
    hipMemcpy(seed, h, sizeof h, hipMemcpyHostToDevice);
    const double f32 = 2.0 * 32 * 32 * 64, f16 = 2.0 * 16 * 16 * 128;
    for (int w : {1, 2, 4}) {
        run("32x32x64", k32<1>, f32, 1, w, seed, out);
        run("32x32x64", k32<2>, f32, 2, w, seed, out);
        run("32x32x64", k32<4>, f32, 4, w, seed, out);
        run("32x32x64 scaled", k32<1, true>, f32, 1, w, seed, out);
        run("32x32x64 scaled", k32<4, true>, f32, 4, w, seed, out);
        run("16x16x128", k16<1>, f16, 1, w, seed, out);
        run("16x16x128", k16<4>, f16, 4, w, seed, out);
    }
    return 0;
}
