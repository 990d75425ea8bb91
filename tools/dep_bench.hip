// VALU issue model on gfx950: K independent dependent-chains of v_add_f32 per lane,
// W waves per SIMD (occupancy pinned with dynamic LDS: one 256-thread workgroup = one
// wave per SIMD, W workgroups per CU). Prints cycles per wave-instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/dep_bench.hip -o build/dep_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;

template <int K, int OP>
__global__ __launch_bounds__(256) void chains(float* out, float seed) {
    extern __shared__ float lds[];
    float v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = seed + threadIdx.x + k;
    const float w = seed * 0.5f;
    float u[K];
#pragma unroll
    for (int k = 0; k < K; ++k) u[k] = seed * (0.25f + k);
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[k]) : "v"(w));
            if (OP == 1) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(v[k]) : "v"(w));
            if (OP == 2) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(*(double*)&v[k & ~1]) : "v"(*(double*)&v[0]));
            if (OP == 3) asm volatile("v_add_f32 %0, 0x4b400000, %0" : "+v"(v[k]));
            if (OP == 4) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(v[k]) : "v"(w), "v"(u[k]));
            if (OP == 5) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[k]) : "v"(u[k]));
            if (OP == 6) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[k]) : "v"(u[k]), "v"(u[(k + 1) % K]));
            if (OP == 7) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[k]) : "v"(u[k]));
        }
    }
    float s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += v[k];
    if (s == 12345.f) lds[threadIdx.x] = s, out[threadIdx.x] = lds[threadIdx.x ^ 1];
}

template <int K, int OP>
void run(const char* name, float* out, int cus, int wps) {
    const size_t lds = (160 * 1024) / wps - 1024;
    hipFuncSetAttribute((const void*)chains<K, OP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int grid = cus * wps * 8;  // 8 rounds of resident workgroups
    hipLaunchKernelGGL((chains<K, OP>), dim3(grid), dim3(256), lds, 0, out, 1.f);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"error\": \"launch (lds %zu)\"}\n", name, K, wps, lds);
        return;
    }
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        hipEventRecord(a);
        hipLaunchKernelGGL((chains<K, OP>), dim3(grid), dim3(256), lds, 0, out, 1.f + r);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    // wave-instructions per SIMD: grid*4 waves / (cus*4 SIMDs) * ITERS * K
    const double wi = (double)grid * 4 / (cus * 4.0) * ITERS * K;
    const double ns_per = best * 1e6 / wi;
    printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ns_per_wave_instr\": %.3f, "
           "\"cycles_at_2.4GHz\": %.2f}\n", name, K, wps, ns_per, ns_per * 2.4);
    fflush(stdout);
}

template <int OP>
void sweep(const char* name, float* out, int cus) {
    for (int w : {2, 4, 8}) {
        run<1, OP>(name, out, cus, w);
        run<2, OP>(name, out, cus, w);
        run<4, OP>(name, out, cus, w);
        run<8, OP>(name, out, cus, w);
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    float* out;
    hipMalloc(&out, 4096);
    sweep<4>("v_fmac_f32 w,u[k]", out, p.multiProcessorCount);
    sweep<5>("v_mul_f32 v,u[k]", out, p.multiProcessorCount);
    sweep<6>("v_fma_f32 u[k],u[k+1],v", out, p.multiProcessorCount);
    sweep<7>("v_add_f32 v,u[k]", out, p.multiProcessorCount);
    return 0;
}
