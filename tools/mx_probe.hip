// mx_probe.hip -- checks the gfx950 FP4 (e2m1) MFMA operand maps and the exactness of the
// Hamming-key encoding used by the MFMA search (kernels.hip search_mx_kernel):
//   D = A * B + C, A = right-descriptor bits {0, 1}, B = 1 - 2*left bits {+1, -1},
//   C = col1 * 2^-15  ->  D = (ham - |left|) + col1 * 2^-15, exact in f32.
// Host packs operands under the assumed lane maps and compares against a double-precision
// GEMM; prints PASS/FAIL per shape. Build: hipcc --offload-arch=gfx950 -O2 mx_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cmath>
#include <vector>
#include <random>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void mfma32(const int* a, const int* b, const float* c, float* d, int chain) {
    int l = threadIdx.x;
    v16f acc;
    for (int r = 0; r < 16; ++r) acc[r] = c[l * 16 + r];
    for (int s = 0; s < chain; ++s) {
        v8i av = {a[(s * 64 + l) * 4 + 0], a[(s * 64 + l) * 4 + 1], a[(s * 64 + l) * 4 + 2], a[(s * 64 + l) * 4 + 3], 0, 0, 0, 0};
        v8i bv = {b[(s * 64 + l) * 4 + 0], b[(s * 64 + l) * 4 + 1], b[(s * 64 + l) * 4 + 2], b[(s * 64 + l) * 4 + 3], 0, 0, 0, 0};
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 4, 4, 0, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) d[l * 16 + r] = acc[r];
}

__global__ void mfma16(const int* a, const int* b, const float* c, float* d, int chain) {
    int l = threadIdx.x;
    v4f acc;
    for (int r = 0; r < 4; ++r) acc[r] = c[l * 4 + r];
    for (int s = 0; s < chain; ++s) {
        v8i av = {a[(s * 64 + l) * 4 + 0], a[(s * 64 + l) * 4 + 1], a[(s * 64 + l) * 4 + 2], a[(s * 64 + l) * 4 + 3], 0, 0, 0, 0};
        v8i bv = {b[(s * 64 + l) * 4 + 0], b[(s * 64 + l) * 4 + 1], b[(s * 64 + l) * 4 + 2], b[(s * 64 + l) * 4 + 3], 0, 0, 0, 0};
        acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 4, 4, 0, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}

static int code(int v) { return v == 0 ? 0 : v == 1 ? 0x2 : v == -1 ? 0xA : (abort(), 0); }

// shape: M=N=32, K=64 per step (32x32x64) or M=N=16, K=128 (16x16x128)
static int run(bool big, int chain, int mode, std::mt19937& rng) {
    const int MN = big ? 32 : 16, KS = big ? 64 : 128, K = KS * chain;
    const int KPL = 32;  // fp4 elements per lane per step
    std::vector<int> A(MN * K), B(K * MN);
    std::vector<double> C(MN * MN);
    for (auto& v : A) v = (mode == 1) ? 1 : (int)(rng() & 1);
    for (auto& v : B) v = (mode == 1) ? -1 : ((rng() & 1) ? 1 : -1);
    for (int i = 0; i < MN; ++i)
        for (int j = 0; j < MN; ++j) C[i * MN + j] = (double)((i * 977 + j * 131 + 4000) % 32768) / 32768.0;
    std::vector<int> pa(chain * 64 * 4, 0), pb(chain * 64 * 4, 0);
    for (int s = 0; s < chain; ++s)
        for (int l = 0; l < 64; ++l) {
            int row = big ? (l & 31) : (l & 15);
            int kb = s * KS + (big ? 32 * (l >> 5) : 32 * (l >> 4));
            for (int j = 0; j < KPL; ++j) {
                int q = j / 8, p = j % 8;
                pa[(s * 64 + l) * 4 + q] |= code(A[row * K + kb + j]) << (4 * p);
                pb[(s * 64 + l) * 4 + q] |= code(B[(kb + j) * MN + row]) << (4 * p);
            }
        }
    const int R = big ? 16 : 4;
    std::vector<float> pc(64 * R), pd(64 * R);
    auto rowof = [&](int l, int r) { return big ? (r & 3) + 8 * (r >> 2) + 4 * (l >> 5) : 4 * (l >> 4) + r; };
    auto colof = [&](int l) { return big ? (l & 31) : (l & 15); };
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < R; ++r) pc[l * R + r] = (float)C[rowof(l, r) * MN + colof(l)];
    int *da, *db; float *dc, *dd;
    hipMalloc(&da, pa.size() * 4); hipMalloc(&db, pb.size() * 4);
    hipMalloc(&dc, pc.size() * 4); hipMalloc(&dd, pd.size() * 4);
    hipMemcpy(da, pa.data(), pa.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, pb.data(), pb.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dc, pc.data(), pc.size() * 4, hipMemcpyHostToDevice);
    if (big) mfma32<<<1, 64>>>(da, db, dc, dd, chain); else mfma16<<<1, 64>>>(da, db, dc, dd, chain);
    hipMemcpy(pd.data(), dd, pd.size() * 4, hipMemcpyDeviceToHost);
    hipFree(da); hipFree(db); hipFree(dc); hipFree(dd);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < R; ++r) {
            int i = rowof(l, r), j = colof(l);
            double e = C[i * MN + j];
            for (int k = 0; k < K; ++k) e += (double)A[i * K + k] * B[k * MN + j];
            if ((double)pd[l * R + r] != e) {
                if (bad < 4) printf("  mismatch lane %d reg %d (row %d col %d): got %.9g want %.9g\n", l, r, i, j, pd[l * R + r], e);
                ++bad;
            }
        }
    printf("%s chain=%d mode=%d: %s (%d bad of %d)\n", big ? "32x32x64" : "16x16x128", chain, mode,
           bad ? "FAIL" : "PASS", bad, 64 * R);
    return bad;
}

int main() {
    std::mt19937 rng(1234);
    int bad = 0;
    for (int mode = 0; mode < 2; ++mode)
        for (int chain = 1; chain <= 4; chain *= 2) {
            bad += run(true, chain, mode, rng);
            bad += run(false, chain, mode, rng);
        }
    printf(bad ? "MX PROBE FAIL\n" : "MX PROBE PASS\n");
    return bad ? 1 : 0;
}
