// Does VALU work of one wave overlap the FP4 MFMAs (v_mfma_scale_f32_32x32x64_f8f6f4) of
// another wave on the same SIMD, or of the same wave when interleaved? One workgroup of 8 waves
// per CU (2 per SIMD, LDS-limited), modes:
//   0: waves 0-3 MFMA only (the others exit)      1: waves 4-7 VALU only
//   2: both (waves 0-3 MFMA, 4-7 VALU)             3: every wave MFMA + VALU, program order
//      grouped (4 MFMAs, then their 24 VALU)       4: the same work, interleaved per MFMA
//      (sched_group_barrier: 1 MFMA, 6 VALU)
// Prints ms per mode; time(2) ~ max(0, 1) means the pipes overlap across waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v4i_t __attribute__((ext_vector_type(4)));

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
// KIND 0: FP4 with E8M0 scales (v_mfma_scale_f32_32x32x64_f8f6f4), 1: FP4 unscaled
// (v_mfma_f32_32x32x64_f8f6f4), 2: bf16 (v_mfma_f32_32x32x16_bf16)
template <int KIND>
__device__ __forceinline__ v16f mm(v8i a, v8i b, v16f c, int sa) {
    if constexpr (KIND == 0)
        return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, sa, 0, 127);
    else if constexpr (KIND == 1)
        return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, (v4i_t){a[0], a[1], a[2], a[3]}),
                                                       __builtin_bit_cast(v8bf, (v4i_t){b[0], b[1], b[2], b[3]}), c, 0, 0, 0);
}

template <int MODE, int KIND>
__global__ __launch_bounds__(512) void k(float* out, int iters) {
    extern __shared__ int lds[];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const bool do_mfma = MODE == 0 ? wave < 4 : MODE == 1 ? false : MODE == 2 ? wave < 4 : true;
    const bool do_valu = MODE == 0 ? false : MODE == 1 ? wave >= 4 : MODE == 2 ? wave >= 4 : true;
    if (!do_mfma && !do_valu) return;
    v8i a = {lane, lane + 1, lane * 3, 7, 0, 0, 0, 0};
    v8i b = {lane ^ 5, 3, lane, 1, 0, 0, 0, 0};
    v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
    uint32_t x[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) x[i] = lane * 7 + i;
    const int sa = 127 - (lane & 1);
    for (int it = 0; it < iters; ++it) {
        if (MODE <= 2) {
            if (do_mfma) {
                c0 = mm<KIND>(a, b, c0, sa);
                c1 = mm<KIND>(a, b, c1, sa);
                c2 = mm<KIND>(a, b, c2, sa);
                c3 = mm<KIND>(a, b, c3, sa);
            }
            if (do_valu) {
#pragma unroll
                for (int i = 0; i < 24; ++i) x[i] = min(min(x[i], x[(i + 1) % 24] + 1u), x[(i + 5) % 24]);
            }
        } else {
            c0 = mm<KIND>(a, b, c0, sa);
            c1 = mm<KIND>(a, b, c1, sa);
            c2 = mm<KIND>(a, b, c2, sa);
            c3 = mm<KIND>(a, b, c3, sa);
#pragma unroll
            for (int i = 0; i < 24; ++i) x[i] = min(min(x[i], x[(i + 1) % 24] + 1u), x[(i + 5) % 24]);
            if (MODE == 4) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, 12, 0); // then VALU
                }
            }
        }
    }
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    uint32_t t = 0;
    for (int i = 0; i < 24; ++i) t ^= x[i];
    out[blockIdx.x * 512 + threadIdx.x] = s + (float)t + (float)lds[threadIdx.x & 15];
}

template <int MODE, int KIND>
float run(float* out, int iters, int cus) {
    const size_t lds = 100 * 1024;
    hipFuncSetAttribute((const void*)k<MODE, KIND>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((k<MODE, KIND>), dim3(cus), dim3(512), lds, 0, out, iters);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<MODE, KIND>), dim3(cus), dim3(512), lds, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    int cus = 256;
    float* out;
    hipMalloc(&out, 256 * 512 * 4);
    const int iters = 20000;
    auto cyc = [&](float ms) { return ms * 1e-3 * 2.4e9 / iters; };
    const char* names[3] = {"fp4_scaled", "fp4", "bf16_32x32x16"};
    float t[3][5];
    t[0][0] = run<0, 0>(out, iters, cus); t[0][1] = run<1, 0>(out, iters, cus); t[0][2] = run<2, 0>(out, iters, cus);
    t[0][3] = run<3, 0>(out, iters, cus); t[0][4] = run<4, 0>(out, iters, cus);
    t[1][0] = run<0, 1>(out, iters, cus); t[1][1] = run<1, 1>(out, iters, cus); t[1][2] = run<2, 1>(out, iters, cus);
    t[1][3] = run<3, 1>(out, iters, cus); t[1][4] = run<4, 1>(out, iters, cus);
    t[2][0] = run<0, 2>(out, iters, cus); t[2][1] = run<1, 2>(out, iters, cus); t[2][2] = run<2, 2>(out, iters, cus);
    t[2][3] = run<3, 2>(out, iters, cus); t[2][4] = run<4, 2>(out, iters, cus);
    for (int k = 0; k < 3; ++k)
        printf("{\"mfma\": \"%s\", \"unit\": \"cycles per iteration and SIMD (4 MFMA, 24 v_min3 + 24 v_add)\", "
               "\"mfma_wave_only\": %.1f, \"valu_wave_only\": %.1f, \"both_waves\": %.1f, "
               "\"same_wave\": %.1f, \"same_wave_interleaved\": %.1f}\n",
               names[k], cyc(t[k][0]), cyc(t[k][1]), cyc(t[k][2]), cyc(t[k][3]), cyc(t[k][4]));
    return 0;
}
