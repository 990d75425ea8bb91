// search_variants.hip -- standalone A/B harness for formulations of the 128-bit packed
// search inner loop (the library's search16_kernel<4, NODUPES, 1> structure: whole right
// row in LDS, 2 col0 per lane, 16-bit packed keys, 256-column tiles).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/search_variants.hip -o build/search_variants
//   build/search_variants [rows=1536] [cols=2048] [waves=8]
// Every variant's output is compared with variant 0; timings are interleaved rounds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}

// V0: opaque empty asm on the accumulator (library as of this commit)
// V1: like V0 but the seed enters the first bcnt directly (no asm on the seed)
// V2: no asm at all (compiler chooses; expect v_add3)
// V3: whole pair step (xor+bcnt chain x2, perm, pk_min x2, xor) as one asm block
// V4: accumulator made opaque by AND with a runtime all-ones mask (fast v_and)
template <int V>
__device__ __forceinline__ uint32_t ham2(uint4 a, uint4 d, uint32_t seed, uint32_t ones) {
    if (V == 0) {
        uint32_t c = seed;
        asm("" : "+v"(c));
        c = __builtin_popcount(a.x ^ d.x) + c;
        asm("" : "+v"(c));
        c = __builtin_popcount(a.y ^ d.y) + c;
        asm("" : "+v"(c));
        c = __builtin_popcount(a.z ^ d.z) + c;
        asm("" : "+v"(c));
        return __builtin_popcount(a.w ^ d.w) + c;
    } else if (V == 1) {
        uint32_t c = __builtin_popcount(a.x ^ d.x) + seed;
        asm("" : "+v"(c));
        c = __builtin_popcount(a.y ^ d.y) + c;
        asm("" : "+v"(c));
        c = __builtin_popcount(a.z ^ d.z) + c;
        asm("" : "+v"(c));
        return __builtin_popcount(a.w ^ d.w) + c;
    } else if (V == 2) {
        return __builtin_popcount(a.x ^ d.x) + __builtin_popcount(a.y ^ d.y) +
               __builtin_popcount(a.z ^ d.z) + __builtin_popcount(a.w ^ d.w) + seed;
    } else {  // V == 4
        uint32_t c = __builtin_popcount(a.x ^ d.x) + seed;
        c = __builtin_popcount(a.y ^ d.y) + (c & ones);
        c = __builtin_popcount(a.z ^ d.z) + (c & ones);
        return __builtin_popcount(a.w ^ d.w) + (c & ones);
    }
}

template <int V>
__device__ __forceinline__ void step(const uint4 d, uint32_t seed, uint4 a0, uint4 a1, uint32_t& lo,
                                     uint32_t& hi, uint32_t ones) {
    if (V == 3) {
        uint32_t t0, t1, r0, r1;
        asm("v_xor_b32 %[t0], %[d0], %[a0x]\n\t"
            "v_xor_b32 %[t1], %[d0], %[a1x]\n\t"
            "v_bcnt_u32_b32 %[r0], %[t0], %[seed]\n\t"
            "v_bcnt_u32_b32 %[r1], %[t1], %[seed]\n\t"
            "v_xor_b32 %[t0], %[d1], %[a0y]\n\t"
            "v_xor_b32 %[t1], %[d1], %[a1y]\n\t"
            "v_bcnt_u32_b32 %[r0], %[t0], %[r0]\n\t"
            "v_bcnt_u32_b32 %[r1], %[t1], %[r1]\n\t"
            "v_xor_b32 %[t0], %[d2], %[a0z]\n\t"
            "v_xor_b32 %[t1], %[d2], %[a1z]\n\t"
            "v_bcnt_u32_b32 %[r0], %[t0], %[r0]\n\t"
            "v_bcnt_u32_b32 %[r1], %[t1], %[r1]\n\t"
            "v_xor_b32 %[t0], %[d3], %[a0w]\n\t"
            "v_xor_b32 %[t1], %[d3], %[a1w]\n\t"
            "v_bcnt_u32_b32 %[r0], %[t0], %[r0]\n\t"
            "v_bcnt_u32_b32 %[r1], %[t1], %[r1]\n\t"
            "v_perm_b32 %[r0], %[r1], %[r0], %[sel]\n\t"
            "v_pk_min_u16 %[lo], %[lo], %[r0]\n\t"
            "v_xor_b32 %[r0], 0xff00ff, %[r0]\n\t"
            "v_pk_min_u16 %[hi], %[hi], %[r0]"
            : [t0] "=&v"(t0), [t1] "=&v"(t1), [r0] "=&v"(r0), [r1] "=&v"(r1), [lo] "+v"(lo),
              [hi] "+v"(hi)
            : [d0] "v"(d.x), [d1] "v"(d.y), [d2] "v"(d.z), [d3] "v"(d.w), [a0x] "v"(a0.x),
              [a0y] "v"(a0.y), [a0z] "v"(a0.z), [a0w] "v"(a0.w), [a1x] "v"(a1.x), [a1y] "v"(a1.y),
              [a1z] "v"(a1.z), [a1w] "v"(a1.w), [seed] "s"(seed), [sel] "s"(0x04050001u));
        return;
    }
    const uint32_t r0 = ham2<V>(a0, d, seed, ones);
    const uint32_t r1 = ham2<V>(a1, d, seed, ones);
    const uint32_t key = __builtin_amdgcn_perm(r1, r0, 0x04050001u);
    lo = pk_min_u16(lo, key);
    hi = pk_min_u16(hi, key ^ 0x00FF00FFu);
}

template <int V>
__global__ __launch_bounds__(512) void kern(const uint4* __restrict__ d0g, const uint4* __restrict__ d1g,
                                            int rows, int cols, int tiles_per_row, uint32_t ones,
                                            int16_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds[];
    const int bid = blockIdx.x, nwg = gridDim.x, per = (nwg + 7) / 8;
    const int logical = nwg % 8 ? bid : (bid % 8) * per + bid / 8;
    const int row = logical / tiles_per_row, tile = logical % tiles_per_row;
    const int waves = blockDim.x / 64, wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int c0 = tile * waves * 128 + wave * 128 + lane;
    const uint4* r0 = d0g + (size_t)row * cols;
    const uint4* r1 = d1g + (size_t)row * cols;
    for (int i = threadIdx.x; i < cols; i += blockDim.x) lds[i] = r1[i];
    __syncthreads();
    const uint4 a0 = r0[min(c0, cols - 1)], a1 = r0[min(c0 + 64, cols - 1)];
    uint32_t glo0 = ~0u, glo1 = ~0u, ghi0 = ~0u, ghi1 = ~0u;
    for (int t0 = 0; t0 < cols; t0 += 256) {
        const int tn = min(256, cols - t0);
        uint32_t lo = ~0u, hi = ~0u;
        int j = 0;
        for (; j + 8 <= tn; j += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) step<V>(lds[t0 + j + u], (uint32_t)(j + u) << 8, a0, a1, lo, hi, ones);
        }
        for (; j < tn; ++j) step<V>(lds[t0 + j], (uint32_t)j << 8, a0, a1, lo, hi, ones);
        const uint32_t tb = t0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t v = (lo >> (16 * h)) & 0xFFFFu, w = (hi >> (16 * h)) & 0xFFFFu;
            const uint32_t k = ((v >> 8) << 16) | (tb + (v & 0xFFu));
            const uint32_t last = tb + 255u - (w & 0xFFu);
            const uint32_t kh = ((w >> 8) << 16) | (0xFFFFu - last);
            if (h == 0) { glo0 = min(glo0, k); ghi0 = min(ghi0, kh); }
            else { glo1 = min(glo1, k); ghi1 = min(ghi1, kh); }
        }
    }
    int16_t* o = out + (size_t)row * cols;
    if (c0 < cols) {
        const int f = glo0 & 0xFFFF;
        o[c0] = (0xFFFF - (ghi0 & 0xFFFF)) != (uint32_t)f ? (int16_t)-32768 : (int16_t)(c0 - f);
    }
    if (c0 + 64 < cols) {
        const int f = glo1 & 0xFFFF;
        o[c0 + 64] = (0xFFFF - (ghi1 & 0xFFFF)) != (uint32_t)f ? (int16_t)-32768 : (int16_t)(c0 + 64 - f);
    }
}

typedef void (*kfn)(const uint4*, const uint4*, int, int, int, uint32_t, int16_t*);

int main(int argc, char** argv) {
    const int rows = argc > 1 ? atoi(argv[1]) : 1536;
    const int cols = argc > 2 ? atoi(argv[2]) : 2048;
    const int waves = argc > 3 ? atoi(argv[3]) : 8;
    std::vector<uint4> h0((size_t)rows * cols), h1((size_t)rows * cols);
    uint64_t s = 0x600DF00D;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 32); };
    for (size_t i = 0; i < h0.size(); ++i) {
        h0[i] = make_uint4(rnd(), rnd(), rnd(), rnd() & 0x3FFFFFFF);
    }
    for (int r = 0; r < rows; ++r)  // right row = left row shifted by 16..63 with a few flips
        for (int c = 0; c < cols; ++c) {
            int src = std::min(cols - 1, c + 16 + (r * 48) / rows);
            uint4 v = h0[(size_t)r * cols + src];
            if (rnd() % 4 == 0) v.x ^= 1u << (rnd() % 32);
            h1[(size_t)r * cols + c] = v;
        }
    uint4 *d0, *d1;
    int16_t* out;
    CHECK(hipMalloc(&d0, h0.size() * 16));
    CHECK(hipMalloc(&d1, h1.size() * 16));
    CHECK(hipMalloc(&out, (size_t)rows * cols * 2 * 5));
    CHECK(hipMemcpy(d0, h0.data(), h0.size() * 16, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d1, h1.data(), h1.size() * 16, hipMemcpyHostToDevice));
    const int tpr = (cols + waves * 128 - 1) / (waves * 128);
    const int nwg = rows * tpr;
    kfn fns[5] = {kern<0>, kern<1>, kern<2>, kern<3>, kern<4>};
    const char* names[5] = {"V0 asm-opaque acc", "V1 seed direct", "V2 no asm", "V3 full asm step",
                            "V4 and-mask"};
    std::vector<std::vector<float>> t(5);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int rnd_ = 0; rnd_ < 7; ++rnd_)
        for (int v = 0; v < 5; ++v) {
            CHECK(hipEventRecord(a));
            for (int k = 0; k < 5; ++k)
                hipLaunchKernelGGL(fns[v], dim3(nwg), dim3(64 * waves), cols * 16, 0, d0, d1, rows,
                                   cols, tpr, 0xFFFFFFFFu, out + (size_t)v * rows * cols);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            t[v].push_back(ms / 5);
        }
    std::vector<int16_t> ho((size_t)rows * cols * 5);
    CHECK(hipMemcpy(ho.data(), out, ho.size() * 2, hipMemcpyDeviceToHost));
    const double pairs = (double)rows * cols * cols;
    for (int v = 0; v < 5; ++v) {
        bool same = std::equal(ho.begin(), ho.begin() + (size_t)rows * cols,
                               ho.begin() + (size_t)v * rows * cols);
        std::sort(t[v].begin(), t[v].end());
        printf("{\"variant\": \"%s\", \"ms_median\": %.4f, \"ms_min\": %.4f, \"Gpairs_s\": %.1f, "
               "\"same_as_V0\": %s}\n",
               names[v], t[v][3], t[v][0], pairs / (t[v][3] * 1e-3) / 1e9, same ? "true" : "false");
    }
    long valid = 0;
    for (size_t i = 0; i < (size_t)rows * cols; ++i) valid += ho[i] != -32768;
    printf("{\"valid_frac\": %.4f}\n", (double)valid / ((double)rows * cols));
    return 0;
}
