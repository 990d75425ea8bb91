/*
 * bicos_oracle.c -- TEST INFRASTRUCTURE ONLY (see bicos_oracle.h for the
 * parity status and the reason this file exists). Plain-C restatement of the
 * reference CPU path; every function cites the reference file:line it follows.
 *
 * Build: oracle/Makefile  (gcc -O3 -ffp-contract=off -- the reference's own
 * as-shipped flags do not contract either).
 */
#include "bicos_oracle.h"

#include <limits.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define MAX_N 256

/* ---------------------------------------------------------------- threads */

typedef void (*row_fn)(void* ctx, int row_begin, int row_end);

typedef struct {
    row_fn fn;
    void* ctx;
    int begin, end;
} row_job;

static void* row_job_main(void* p) {
    row_job* j = (row_job*)p;
    j->fn(j->ctx, j->begin, j->end);
    return NULL;
}

/* Row-parallel map; stands in for cv::parallel_for_ over rows (every stage of
 * the reference is row-local, so the partition cannot change results). */
static void parallel_rows(int rows, int nthreads, row_fn fn, void* ctx) {
    if (nthreads <= 1 || rows < 2) {
        fn(ctx, 0, rows);
        return;
    }
    if (nthreads > rows) nthreads = rows;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    row_job jobs[256];
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].fn = fn;
        jobs[i].ctx = ctx;
        jobs[i].begin = (int)((long)rows * i / nthreads);
        jobs[i].end = (int)((long)rows * (i + 1) / nthreads);
        pthread_create(&th[i], NULL, row_job_main, &jobs[i]);
    }
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
}

static inline unsigned pix_at(const void* stack, int depth, size_t idx) {
    return depth == 1 ? ((const uint8_t*)stack)[idx] : ((const uint16_t*)stack)[idx];
}

/* ------------------------------------------------------------- dispatch */

/* src/impl/cpu.cpp:122-124 */
int bicos_oracle_required_bits(int n, int mode) {
    return mode == 1 ? n * n - 2 * n + 3 : 4 * n - 7;
}

/* src/impl/cpu.cpp:129-156: <=32 -> uint32, <=64 -> uint64, <=128 -> uint128,
 * <=256 -> bitset<256>, else std::invalid_argument. Returned in uint32 words. */
int bicos_oracle_desc_words(int n, int mode) {
    int bits = bicos_oracle_required_bits(n, mode);
    if (bits < 0) return -1;
    if (bits <= 32) return 1;
    if (bits <= 64) return 2;
    if (bits <= 128) return 4;
    if (bits <= 256) return 8;
    return -1;
}

/* ------------------------------------------------------------ transform */

typedef struct {
    uint32_t* v;
    int words;
    unsigned i;
} bitwriter;

/* include/impl/cpu/bitfield.hpp:34-58: bit i := i-th comparison, LSB first. */
static inline void bw_set(bitwriter* bw, int value) {
    if (value && (int)(bw->i / 32) < bw->words) bw->v[bw->i / 32] |= 1u << (bw->i % 32);
    bw->i++;
}

/* include/impl/cpu/descriptor_transform.hpp:31-73 (transform_limited) */
static void transform_limited_px(const unsigned* pix, int n, uint32_t* out, int words) {
    bitwriter bf = {out, words, 0};
    memset(out, 0, sizeof(uint32_t) * words);

    float av = 0.0f;
    for (int t = 0; t < n; ++t) av += (float)pix[t];
    av /= (float)n;

    int prev_pair_sums[2] = {-1, -1};
    for (int t = 0; t < n - 2; ++t) {
        const unsigned a = pix[t], b = pix[t + 1], c = pix[t + 2];
        bw_set(&bf, a < b);
        bw_set(&bf, a < c);
        bw_set(&bf, (float)a < av);
        int* prev = &prev_pair_sums[t % 2];
        const int cur = (int)(a + b);
        if (*prev != -1) bw_set(&bf, *prev < cur);
        *prev = cur;
    }
    const unsigned a = pix[n - 2], b = pix[n - 1];
    bw_set(&bf, a < b);
    bw_set(&bf, (float)a < av);
    bw_set(&bf, (float)b < av);
    bw_set(&bf, prev_pair_sums[(n - 2) % 2] < (int)(a + b));
}

/* include/impl/cpu/descriptor_transform.hpp:75-123 (transform_full) */
static void transform_full_px(const unsigned* pix, int n, uint32_t* out, int words) {
    bitwriter bf = {out, words, 0};
    memset(out, 0, sizeof(uint32_t) * words);

    float av = 0.0f;
    for (int t = 0; t < n; ++t) av += (float)pix[t];
    av /= (float)n;

    unsigned pairsums[MAX_N];
    for (int t = 0; t < n - 2; ++t) {
        const unsigned a = pix[t], b = pix[t + 1], c = pix[t + 2];
        bw_set(&bf, a < b);
        bw_set(&bf, a < c);
        bw_set(&bf, (float)a < av);
        pairsums[t] = pix[t] + pix[t + 1];
    }
    pairsums[n - 2] = pix[n - 2] + pix[n - 1];

    const unsigned a = pix[n - 2], b = pix[n - 1];
    bw_set(&bf, a < b);
    bw_set(&bf, (float)a < av);
    bw_set(&bf, (float)b < av);

    for (int t = 0; t < n - 1; ++t)
        for (int i = 0; i < n - 1; ++i) {
            if (i == t || i == t - 1 || i == t + 1) continue;
            bw_set(&bf, pairsums[t] < pairsums[i]);
        }
}

typedef struct {
    const void* stack;
    int n, rows, cols, depth, mode, words;
    uint32_t* desc;
} transform_ctx;

/* include/impl/cpu/descriptor_transform.hpp:125-138 */
static void transform_rows(void* p, int r0, int r1) {
    transform_ctx* c = (transform_ctx*)p;
    const size_t plane = (size_t)c->rows * c->cols;
    unsigned pix[MAX_N];
    for (int r = r0; r < r1; ++r)
        for (int col = 0; col < c->cols; ++col) {
            const size_t idx = (size_t)r * c->cols + col;
            for (int t = 0; t < c->n; ++t) pix[t] = pix_at(c->stack, c->depth, t * plane + idx);
            uint32_t* out = c->desc + idx * c->words;
            if (c->mode == 1)
                transform_full_px(pix, c->n, out, c->words);
            else
                transform_limited_px(pix, c->n, out, c->words);
        }
}

void bicos_oracle_transform(const void* stack, int n, int rows, int cols, int depth, int mode,
                            int words, uint32_t* desc, int nthreads) {
    transform_ctx c = {stack, n, rows, cols, depth, mode, words, desc};
    parallel_rows(rows, nthreads, transform_rows, &c);
}

/* --------------------------------------------------------------- search */

/* include/impl/cpu/bicos.hpp:29-48 (ham) */
static inline int ham(const uint32_t* a, const uint32_t* b, int words) {
    int c = 0;
    switch (words) {
        case 1:
            return __builtin_popcount(a[0] ^ b[0]);
        case 2: {
            uint64_t x, y;
            memcpy(&x, a, 8);
            memcpy(&y, b, 8);
            return __builtin_popcountll(x ^ y);
        }
        default:
            for (int w = 0; w < words; w += 2) {
                uint64_t x, y;
                memcpy(&x, a + w, 8);
                memcpy(&y, b + w, 8);
                c += __builtin_popcountll(x ^ y);
            }
            return c;
    }
}

#define INVALID_INT INT_MIN        /* INVALID_DISP<int> = numeric_limits<int>::lowest() */
#define INVALID_I16 ((int16_t)-32768)

/* include/impl/cpu/bicos.hpp:50-76 (bicos_search): full-row argmin, strict '<' so the
 * lowest col1 wins ties; with NODUPES the result is invalid iff the minimum is attained
 * more than once. */
static int bicos_search(const uint32_t* d0, const uint32_t* row1, int cols, int words, int flags) {
    int best_col1 = INVALID_INT, min_cost = INT_MAX, dupes = 0;
    for (int col1 = 0; col1 < cols; ++col1) {
        const int cost = ham(d0, row1 + (size_t)col1 * words, words);
        if (cost < min_cost) {
            min_cost = cost;
            best_col1 = col1;
            if (flags & BICOS_ORACLE_NODUPES) dupes = 0;
        } else if ((flags & BICOS_ORACLE_NODUPES) && cost == min_cost) {
            dupes++;
        }
    }
    if ((flags & BICOS_ORACLE_NODUPES) && dupes > 0) return INVALID_INT;
    return best_col1;
}

typedef struct {
    const uint32_t *d0, *d1;
    int rows, cols, words, flags, max_lr_diff;
    int16_t* out;
} search_ctx;

/* include/impl/cpu/bicos.hpp:78-113 (bicos) */
static void search_rows(void* p, int r0, int r1) {
    search_ctx* c = (search_ctx*)p;
    for (int r = r0; r < r1; ++r) {
        const uint32_t* row0 = c->d0 + (size_t)r * c->cols * c->words;
        const uint32_t* row1 = c->d1 + (size_t)r * c->cols * c->words;
        int16_t* out = c->out + (size_t)r * c->cols;
        for (int col0 = 0; col0 < c->cols; ++col0) {
            out[col0] = INVALID_I16;
            const int best = bicos_search(row0 + (size_t)col0 * c->words, row1, c->cols, c->words,
                                          c->flags);
            if (best == INVALID_INT) continue;
            if (c->flags & BICOS_ORACLE_CONSISTENCY) {
                const int rev = bicos_search(row1 + (size_t)best * c->words, row0, c->cols,
                                             c->words, c->flags);
                if (rev == INVALID_INT || abs(col0 - rev) > c->max_lr_diff) continue;
                out[col0] = (int16_t)((col0 + rev) / 2 - best);
            } else {
                out[col0] = (int16_t)(col0 - best);
            }
        }
    }
}

void bicos_oracle_search(const uint32_t* desc0, const uint32_t* desc1, int rows, int cols,
                         int words, int flags, int max_lr_diff, int16_t* disp, int nthreads) {
    search_ctx c = {desc0, desc1, rows, cols, words, flags, max_lr_diff, disp};
    parallel_rows(rows, nthreads, search_rows, &c);
}

/* ---------------------------------------------------------------- agree */

/* include/impl/cpu/agree.hpp:28-51 (nxcorr). Float, sequential sums, fmaf
 * accumulators in t order, IEEE division and sqrt. */
static float nxcorr_vals(const unsigned* pix0, const unsigned* pix1, int n, int has_minvar,
                         float minvar) {
    float mean0 = 0.f, mean1 = 0.f;
    for (int i = 0; i < n; ++i) {
        mean0 += (float)pix0[i];
        mean1 += (float)pix1[i];
    }
    mean0 /= (float)n;
    mean1 /= (float)n;

    float covar = 0.f, var0 = 0.f, var1 = 0.f;
    for (int i = 0; i < n; ++i) {
        const float diff0 = (float)pix0[i] - mean0, diff1 = (float)pix1[i] - mean1;
        covar = fmaf(diff0, diff1, covar);
        var0 = fmaf(diff0, diff0, var0);
        var1 = fmaf(diff1, diff1, var1);
    }
    if (has_minvar && (var0 < minvar || var1 < minvar)) return -1.f;
    return covar / sqrtf(var0 * var1);
}

float bicos_oracle_nxcorr(const void* pix0, const void* pix1, int n, int depth, int has_minvar,
                          float minvar_scaled) {
    unsigned a[MAX_N], b[MAX_N];
    for (int i = 0; i < n; ++i) {
        a[i] = pix_at(pix0, depth, i);
        b[i] = pix_at(pix1, depth, i);
    }
    return nxcorr_vals(a, b, n, has_minvar, minvar_scaled);
}

typedef struct {
    int16_t* disp_rw;
    const int16_t* disp_ro;
    const void *s0, *s1;
    int n, rows, cols, depth;
    float thr, step;
    int has_minvar;
    float minvar;
    float* out;
    float* corrmap;
} agree_ctx;

static inline void load_px(const void* s, int depth, size_t plane, size_t idx, int n,
                           unsigned* dst) {
    for (int t = 0; t < n; ++t) dst[t] = pix_at(s, depth, t * plane + idx);
}

/* include/impl/cpu/agree.hpp:53-93 (agree): invalidates int16 disparities in place.
 * corrmap is written for every in-range bicos-valid pixel; a NaN correlation passes
 * the threshold ('nan < thr' is false). */
static void agree_rows(void* p, int r0, int r1) {
    agree_ctx* c = (agree_ctx*)p;
    const size_t plane = (size_t)c->rows * c->cols;
    unsigned a[MAX_N], b[MAX_N];
    for (int r = r0; r < r1; ++r)
        for (int col = 0; col < c->cols; ++col) {
            int16_t* d = &c->disp_rw[(size_t)r * c->cols + col];
            if (*d == INVALID_I16) continue;
            const int idx1 = col - *d;
            if (idx1 < 0 || c->cols <= idx1) {
                *d = INVALID_I16;
                continue;
            }
            load_px(c->s0, c->depth, plane, (size_t)r * c->cols + col, c->n, a);
            load_px(c->s1, c->depth, plane, (size_t)r * c->cols + idx1, c->n, b);
            const float nxc = nxcorr_vals(a, b, c->n, c->has_minvar, c->minvar);
            if (c->corrmap) c->corrmap[(size_t)r * c->cols + col] = nxc;
            if (nxc < c->thr) *d = INVALID_I16;
        }
}

void bicos_oracle_agree(int16_t* disp, const void* stack0, const void* stack1, int n, int rows,
                        int cols, int depth, float threshold, int has_minvar, float minvar_scaled,
                        float* corrmap, int nthreads) {
    agree_ctx c = {disp, NULL, stack0, stack1, n, rows, cols, depth, threshold, 0.f,
                   has_minvar, minvar_scaled, NULL, corrmap};
    parallel_rows(rows, nthreads, agree_rows, &c);
}

/* (TInput)roundevenf(v): g++ lowers the narrowing through a 32-bit integer
 * conversion, so out-of-range values wrap. */
static inline unsigned narrow_input(float v, int depth) {
    const int i = (int)rintf(v);
    return depth == 1 ? (unsigned)(uint8_t)i : (unsigned)(uint16_t)i;
}

/* include/impl/cpu/agree.hpp:95-191 (agree_subpixel) */
static void subpixel_rows(void* p, int r0, int r1) {
    agree_ctx* c = (agree_ctx*)p;
    const size_t plane = (size_t)c->rows * c->cols;
    const int n = c->n;
    unsigned left[MAX_N], y0[MAX_N], y1[MAX_N], y2[MAX_N], interp[MAX_N];
    float A[MAX_N], B[MAX_N], C[MAX_N];
    for (int r = r0; r < r1; ++r)
        for (int col = 0; col < c->cols; ++col) {
            const size_t o = (size_t)r * c->cols + col;
            c->out[o] = NAN;
            const int16_t d = c->disp_ro[o];
            if (d == INVALID_I16) continue;
            const int col1 = col - d;
            if (col1 < 0 || c->cols <= col1) continue;

            load_px(c->s0, c->depth, plane, o, n, left);
            if (col1 == 0 || col1 == c->cols - 1) {
                load_px(c->s1, c->depth, plane, (size_t)r * c->cols + col1, n, y1);
                const float nxc = nxcorr_vals(left, y1, n, c->has_minvar, c->minvar);
                if (c->corrmap) c->corrmap[o] = nxc;
                if (nxc < c->thr) continue;
                c->out[o] = (float)d;
                continue;
            }
            load_px(c->s1, c->depth, plane, (size_t)r * c->cols + col1 - 1, n, y0);
            load_px(c->s1, c->depth, plane, (size_t)r * c->cols + col1, n, y1);
            load_px(c->s1, c->depth, plane, (size_t)r * c->cols + col1 + 1, n, y2);
            for (int t = 0; t < n; ++t) {
                /* 0.5f * ( y0[t] - 2.0f * y1[t] + y2[t]) ; 0.5f * (-y0[t] + y2[t]) ; y1[t] */
                A[t] = 0.5f * (((float)y0[t] - 2.0f * (float)y1[t]) + (float)y2[t]);
                B[t] = 0.5f * (float)(-(int)y0[t] + (int)y2[t]);
                C[t] = (float)y1[t];
            }
            float best_x = 0.f, best_nxc = -1.f;
            for (float x = -1.f; x <= 1.f; x += c->step) {
                for (int t = 0; t < n; ++t) {
                    const float ax = A[t] * x;
                    const float axx = ax * x;
                    const float bx = B[t] * x;
                    interp[t] = narrow_input((axx + bx) + C[t], c->depth);
                }
                const float nxc = nxcorr_vals(left, interp, n, c->has_minvar, c->minvar);
                if (best_nxc < nxc) {
                    best_x = x;
                    best_nxc = nxc;
                }
            }
            if (c->corrmap) c->corrmap[o] = best_nxc;
            if (best_nxc < c->thr) continue;
            c->out[o] = (float)d - best_x;
        }
}

void bicos_oracle_agree_subpixel(const int16_t* disp, const void* stack0, const void* stack1,
                                 int n, int rows, int cols, int depth, float threshold, float step,
                                 int has_minvar, float minvar_scaled, float* out, float* corrmap,
                                 int nthreads) {
    agree_ctx c = {NULL, disp, stack0, stack1, n, rows, cols, depth, threshold, step,
                   has_minvar, minvar_scaled, out, corrmap};
    parallel_rows(rows, nthreads, subpixel_rows, &c);
}

/* ---------------------------------------------------------------- match */

/* src/impl/cpu.cpp:100-159 (match) + :35-98 (match_impl) */
int bicos_oracle_match(const void* stack0, const void* stack1, int n, int rows, int cols,
                       int depth, const bicos_oracle_config* cfg, void* disp_out, float* corrmap,
                       int nthreads) {
    if (n < 2) return BICOS_ORACLE_ERR_N;
    if (depth != 1 && depth != 2) return BICOS_ORACLE_ERR_DEPTH;
    if (n > MAX_N) return BICOS_ORACLE_ERR_BITS;
    const int words = bicos_oracle_desc_words(n, cfg->mode);
    if (words < 0) return BICOS_ORACLE_ERR_BITS;

    const size_t px = (size_t)rows * cols;
    uint32_t* d0 = (uint32_t*)malloc(px * words * sizeof(uint32_t) + 4);
    uint32_t* d1 = (uint32_t*)malloc(px * words * sizeof(uint32_t) + 4);
    int16_t* raw = (int16_t*)malloc(px * sizeof(int16_t) + 2);

    bicos_oracle_transform(stack0, n, rows, cols, depth, cfg->mode, words, d0, nthreads);
    bicos_oracle_transform(stack1, n, rows, cols, depth, cfg->mode, words, d1, nthreads);

    int flags, lr = -1;
    if (cfg->variant == 1) {
        flags = BICOS_ORACLE_CONSISTENCY | (cfg->no_dupes ? BICOS_ORACLE_NODUPES : 0);
        lr = cfg->max_lr_diff;
    } else {
        flags = BICOS_ORACLE_NODUPES;
    }
    bicos_oracle_search(d0, d1, rows, cols, words, flags, lr, raw, nthreads);
    free(d0);
    free(d1);

    int kind = BICOS_ORACLE_OUT_INT16;
    if (!cfg->has_nxcorr) {
        memcpy(disp_out, raw, px * sizeof(int16_t));
    } else {
        /* cpu.cpp:127: min_var = cfg.min_variance * n (float) */
        const float mv = cfg->has_minvar ? cfg->min_variance * (float)n : 0.f;
        if (corrmap)
            for (size_t i = 0; i < px; ++i) corrmap[i] = NAN; /* cpu.cpp:78-81 */
        if (cfg->has_step) {
            bicos_oracle_agree_subpixel(raw, stack0, stack1, n, rows, cols, depth,
                                        cfg->nxcorr_threshold, cfg->subpixel_step,
                                        cfg->has_minvar, mv, (float*)disp_out, corrmap, nthreads);
        } else {
            bicos_oracle_agree(raw, stack0, stack1, n, rows, cols, depth, cfg->nxcorr_threshold,
                               cfg->has_minvar, mv, corrmap, nthreads);
            float* f = (float*)disp_out; /* cpu.cpp:90-93 convertTo(CV_32F) */
            for (size_t i = 0; i < px; ++i) f[i] = (float)raw[i];
        }
        kind = BICOS_ORACLE_OUT_FLOAT32;
    }
    free(raw);
    return kind;
}
