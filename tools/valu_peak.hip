// valu_peak.hip -- measures the sustained wave64 issue rate of the integer VALU ops the
// BICOS search loop is made of (v_xor_b32, v_bcnt_u32_b32, v_min_u32, v_med3_u32,
// v_lshl_or_b32) on the running MI355X, to price the search kernel's roofline
// against a measured, not assumed, peak. Independent chains, 8 waves/SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o build/valu_peak && build/valu_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHAINS 8
#define ITERS 4096

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
    uint32_t v[CHAINS], w[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
        v[c] = seed * (threadIdx.x + 1) + c;
        w[c] = seed ^ (c * 0x9E3779B9u) ^ blockIdx.x;
    }
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 1) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 2) asm volatile("v_min_u32 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 3) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 4) asm volatile("v_lshl_or_b32 %0, %0, 16, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 5) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "s"(0x05010400u));
            if (OP == 6) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 7) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 8) asm volatile("v_and_b32 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 9) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 10) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 11) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 12) asm volatile("v_min_u32_e64 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 13) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(v[c]) : "s"(seed));
            if (OP == 14) asm volatile("v_mov_b32 %0, %1" : "=v"(v[c]) : "v"(w[c]));
            if (OP == 15) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 17) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 18) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 19) asm volatile("v_cvt_f32_ubyte0 %0, %1" : "=v"(v[c]) : "v"(w[c] ^ v[c]));
            if (OP == 20) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(*(uint64_t*)&v[c & ~1]) : "v"(*(uint64_t*)&w[c & ~1]));
            if (OP == 21) asm volatile("v_rndne_f32 %0, %0" : "+v"(v[c]));
            if (OP == 22) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(v[c]));
            if (OP == 23) asm volatile("v_sub_f32 %0, %1, %0" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 24) asm volatile("v_fma_mix_f32 %0, %1, %0, %0 op_sel_hi:[1,0,0]" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 25) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 26) asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(v[c]) : "v"(w[c] ^ v[c]));
            if (OP == 27) asm volatile("v_or_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 28) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 29) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(*(uint64_t*)&v[c & ~1]) : "v"(*(uint64_t*)&w[c & ~1]));
            if (OP == 30) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 31) asm volatile("v_min_f32 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 32) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 33) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(v[c]), "+v"(w[c]));
            if (OP == 34) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 35) asm volatile("v_min_i32 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 36) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 37) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 38) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 39) asm volatile("v_pk_minimum3_f16 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            if (OP == 40) asm volatile("v_pk_sub_u16 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 41) asm volatile("v_pk_ashrrev_i16 %0, 15, %0" : "+v"(v[c]));
            if (OP == 42) asm volatile("v_pk_min_f16 %0, %0, %1" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 43) asm volatile("v_min3_u16 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "v"(w[(c + 1) % CHAINS]));
            // round 4: 32-bit literal operands (64-bit encodings) vs SGPR / VGPR operands
            if (OP == 44) asm volatile("v_add_f32 %0, 0x4b400000, %0" : "+v"(v[c]));
            if (OP == 45) asm volatile("v_and_b32 %0, 0x4b0000ff, %0" : "+v"(v[c]));
            if (OP == 46) asm volatile("v_add_f32 %0, %1, %0" : "+v"(v[c]) : "s"(seed));
            if (OP == 47 || OP == 48) {  // the subpixel mix per (image, x step): 12 ops, 3 literal (47) or SGPR (48)
                uint32_t a0, a1;
                asm volatile("v_mul_f32 %0, %1, %2" : "=v"(a0) : "v"(w[c]), "v"(v[c]));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a0) : "v"(v[c]));
                asm volatile("v_mul_f32 %0, %1, %2" : "=v"(a1) : "v"(w[(c + 1) % CHAINS]), "v"(v[c]));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a0) : "v"(a1));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a0) : "v"(w[(c + 2) % CHAINS]));
                if (OP == 47) {
                    asm volatile("v_add_f32 %0, 0x4b400000, %0" : "+v"(a0));
                    asm volatile("v_and_b32 %0, 0x4b0000ff, %0" : "+v"(a0));
                    asm volatile("v_add_f32 %0, 0xcb000000, %0" : "+v"(a0));
                } else {
                    asm volatile("v_add_f32 %0, %1, %0" : "+v"(a0) : "s"(0x4b400000u ^ seed));
                    asm volatile("v_and_b32 %0, %1, %0" : "+v"(a0) : "s"(0x4b0000ffu ^ seed));
                    asm volatile("v_add_f32 %0, %1, %0" : "+v"(a0) : "s"(0xcb000000u ^ seed));
                }
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(w[(c + 3) % CHAINS]) : "v"(a0));
                asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a0) : "v"(w[(c + 4) % CHAINS]));
                asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(w[(c + 5) % CHAINS]) : "v"(a0), "v"(w[(c + 6) % CHAINS]));
                asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(w[(c + 7) % CHAINS]) : "v"(a0));
            }
            // round 4: the transform's per-bit pair (compare into an SGPR mask, add-with-carry
            // from it) vs a VGPR-only pair (subtract, then alignbit shifts the sign bit in)
            if (OP == 49) {
                uint64_t m;
                asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(w[c]), "v"(v[c]));
                asm volatile("v_addc_co_u32_e64 %0, vcc, %0, %0, %1" : "+v"(v[c]) : "s"(m) : "vcc");
            }
            if (OP == 50) {
                uint32_t d;
                asm volatile("v_sub_u32 %0, %1, %2" : "=v"(d) : "v"(w[c]), "v"(v[c]));
                asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(v[c]) : "v"(d));
            }
            if (OP == 51) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 52) asm volatile("v_lshrrev_b32 %0, 31, %0" : "+v"(v[c]));
            if (OP == 53) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[c]) : "v"(w[c]));
            if (OP == 54) asm volatile("v_add_u32 %0, %1, %0" : "+v"(v[c]) : "s"(seed));
            if (OP == 55) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(w[c]), "s"(seed));
            if (OP == 56)  // the bit pair through VCC (VOPC e32 + VOP2 add-with-carry)
                asm volatile("v_cmp_lt_u32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
                             : "+v"(v[c]) : "v"(w[c]), "v"(v[c]) : "vcc");
            if (OP == 57) {  // 4 compares into SGPR masks, then 4 adds (the transform's push_lt<4>)
                uint64_t m0, m1, m2, m3, j;
                asm volatile("v_cmp_lt_u32_e64 %1, %6, %7\n\tv_cmp_lt_u32_e64 %2, %6, %8\n\t"
                             "v_cmp_lt_u32_e64 %3, %7, %8\n\tv_cmp_lt_u32_e64 %4, %8, %6\n\t"
                             "v_addc_co_u32_e64 %0, %5, %0, %0, %1\n\tv_addc_co_u32_e64 %0, %5, %0, %0, %2\n\t"
                             "v_addc_co_u32_e64 %0, %5, %0, %0, %3\n\tv_addc_co_u32_e64 %0, %5, %0, %0, %4"
                             : "+v"(v[c]), "=&s"(m0), "=&s"(m1), "=&s"(m2), "=&s"(m3), "=&s"(j)
                             : "v"(w[c]), "v"(w[(c + 1) % CHAINS]), "v"(w[(c + 2) % CHAINS]));
            }
            if (OP == 16) {  // the search loop's 128-bit mix per pair: 4 xor, 4 bcnt, lshl_or, med3, min
                uint32_t t0, t1, t2, t3, cst, key;
                asm volatile("v_xor_b32 %0, %1, %2" : "=v"(t0) : "v"(v[c]), "v"(w[c]));
                asm volatile("v_xor_b32 %0, %1, %2" : "=v"(t1) : "v"(v[c]), "v"(w[(c + 1) % CHAINS]));
                asm volatile("v_xor_b32 %0, %1, %2" : "=v"(t2) : "v"(v[c]), "v"(w[(c + 2) % CHAINS]));
                asm volatile("v_xor_b32 %0, %1, %2" : "=v"(t3) : "v"(v[c]), "v"(w[(c + 3) % CHAINS]));
                asm volatile("v_bcnt_u32_b32 %0, %1, 0" : "=v"(cst) : "v"(t0));
                asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(cst) : "v"(t1));
                asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(cst) : "v"(t2));
                asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(cst) : "v"(t3));
                asm volatile("v_lshl_or_b32 %0, %1, 16, %2" : "=v"(key) : "v"(cst), "s"(i));
                asm volatile("v_med3_u32 %0, %1, %2, %0" : "+v"(w[(c + 4) % CHAINS]) : "v"(v[c]), "v"(key));
                asm volatile("v_min_u32 %0, %0, %1" : "+v"(v[c]) : "v"(key));
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= v[c];
    if (r == 0x12345678u) out[blockIdx.x] = r;
}

template <int OP>
double run(const char* name, uint32_t* out, int grid, int wps = 8) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, out, 3u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, out, 3u + rep);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    const double ops = (double)grid * 256 * ITERS * CHAINS * (OP == 16 ? 11 : (OP == 47 || OP == 48) ? 12 : (OP == 49 || OP == 50 || OP == 56) ? 2 : OP == 57 ? 8 : 1);  // lane-ops
    const double tops = ops / (best * 1e-3) / 1e12;
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"lane_ops\": %.3e, \"ms\": %.4f, \"Tops\": %.2f}\n", name, wps, ops, best, tops);
    return tops;
}

int main(int argc, char** argv) {
    const bool only_new = argc > 1;  // any argument: the ops added in round 2 only
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("{\"device\": \"%s\", \"gcnArch\": \"%s\", \"CUs\": %d, \"clock_khz\": %d, "
           "\"nominal_int32_Tops\": %.2f}\n",
           p.name, p.gcnArchName, p.multiProcessorCount, clk,
           p.multiProcessorCount * 128.0 * clk * 1e3 / 1e12);
    uint32_t* out;
    hipMalloc(&out, 1 << 20);
    const int grid = p.multiProcessorCount * 8 * 4;  // 8 waves/SIMD worth of 256-thr blocks x4
    if (argc > 1 && argv[1][0] == 'l') {  // "lit": literal-operand rates, at 8 and 3 waves/SIMD
        for (int wps : {8, 3}) {
            const int g = p.multiProcessorCount * wps * (wps == 8 ? 4 : 1);
            run<17>("v_add_f32", out, g, wps);
            run<44>("v_add_f32 literal", out, g, wps);
            run<46>("v_add_f32 sgpr", out, g, wps);
            run<8>("v_and_b32", out, g, wps);
            run<45>("v_and_b32 literal", out, g, wps);
            run<47>("subpixel mix 12 ops, 3 literal", out, g, wps);
            run<48>("subpixel mix 12 ops, 3 sgpr", out, g, wps);
        }
        run<49>("v_cmp_lt_u32_e64 sgpr + v_addc_co_u32_e64 (2 ops, transform bit)", out, grid);
        run<50>("v_sub_u32 + v_alignbit_b32 (2 ops)", out, grid);
        run<51>("v_alignbit_b32", out, grid);
        run<52>("v_lshrrev_b32", out, grid);
        run<53>("v_cndmask_b32 vcc", out, grid);
        run<54>("v_add_u32 sgpr", out, grid);
        run<10>("v_min3_u32", out, grid);
        run<55>("v_min3_u32 sgpr", out, grid);
        run<56>("v_cmp_lt_u32_e32 vcc + v_addc_co_u32_e32 vcc (2 ops)", out, grid);
        run<57>("4 x v_cmp_lt_u32_e64 sgpr, then 4 x v_addc_co_u32_e64 (8 ops, push_lt<4>)", out, grid);
        hipFree(out);
        return 0;
    }
    run<39>("v_pk_minimum3_f16", out, grid);
    run<40>("v_pk_sub_u16", out, grid);
    run<41>("v_pk_ashrrev_i16", out, grid);
    run<42>("v_pk_min_f16", out, grid);
    run<43>("v_min3_u16", out, grid);
    run<30>("v_min3_f32", out, grid);
    run<31>("v_min_f32", out, grid);
    run<32>("v_max3_f32", out, grid);
    run<33>("v_permlane32_swap_b32 (per instr)", out, grid);
    run<34>("v_and_or_b32", out, grid);
    run<35>("v_min_i32", out, grid);
    run<36>("v_bfi_b32", out, grid);
    run<37>("v_med3_f32", out, grid);
    run<38>("v_add3_u32", out, grid);
    if (only_new) {
        hipFree(out);
        return 0;
    }
    run<0>("v_xor_b32", out, grid);
    run<1>("v_bcnt_u32_b32", out, grid);
    run<2>("v_min_u32", out, grid);
    run<3>("v_med3_u32", out, grid);
    run<4>("v_lshl_or_b32", out, grid);
    run<5>("v_perm_b32", out, grid);
    run<6>("v_pk_min_u16", out, grid);
    run<7>("v_pk_max_u16", out, grid);
    run<8>("v_and_b32", out, grid);
    run<9>("v_add_u32", out, grid);
    run<10>("v_min3_u32", out, grid);
    run<11>("v_xor_b32_e64", out, grid);
    run<12>("v_min_u32_e64", out, grid);
    run<13>("v_bcnt_u32_b32(sgpr)", out, grid);
    run<14>("v_mov_b32", out, grid);
    run<15>("v_xad_u32", out, grid);
    run<16>("search_mix_128(11 ops/pair)", out, grid);
    run<17>("v_add_f32", out, grid);
    run<18>("v_fmac_f32", out, grid);
    run<19>("v_xor+v_cvt_f32_ubyte0 (2 ops)", out, grid);
    run<20>("v_pk_fma_f32 (per instr)", out, grid);
    run<21>("v_rndne_f32", out, grid);
    run<22>("v_cvt_i32_f32", out, grid);
    run<23>("v_sub_f32", out, grid);
    run<24>("v_fma_mix_f32 (f16 lo operand)", out, grid);
    run<25>("v_pk_add_f16", out, grid);
    run<26>("v_xor+v_cvt_f32_f16 (2 ops)", out, grid);
    run<27>("v_or_b32_sdwa byte0", out, grid);
    run<28>("v_mul_f32", out, grid);
    run<29>("v_pk_mul_f32 (per instr)", out, grid);
    hipFree(out);
    return 0;
}
