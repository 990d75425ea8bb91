/*
 * bicos_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the libBICOS reference CPU path (src/impl/cpu.cpp and
 * include/impl/cpu/{descriptor_transform,bicos,agree}.hpp), written in plain C
 * from the reference's observable semantics. It is the parity CHECKER for the
 * HIP engine in libbicos_amd/ and the "port" CPU baseline timed by bench.py.
 * Nothing in the product path links, loads or calls this code.
 *
 * Parity status: UNPINNED against the reference binary. The reference ships no
 * tests, golden vectors or known-answer fixtures and its CPU
 * path cannot be built in this image without stand-ins for OpenCV headers,
 * which this project does not write. The restatement is instead cross-checked
 * against an independent numpy restatement (oracle/ref_numpy.py), hand-derived
 * known-answer cases and the reference behaviours recorded in SURVEY.md
 * Appendix A (tests/test_oracle.py).
 *
 * Data layout (matches what BICOS::match receives: a vector of n planar images):
 *   stack  : n planes, plane t at stack + t*rows*cols elements, row-major,
 *            element type uint8 (depth 1) or uint16 (depth 2)
 *   desc   : rows*cols descriptors, each `words` uint32 (LSB-first bit i at
 *            word i/32, bit i%32 -- the reference's Bitfield order)
 */
#ifndef BICOS_ORACLE_H
#define BICOS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int has_nxcorr;           /* Config::nxcorr_threshold has_value */
    float nxcorr_threshold;
    int has_step;             /* Config::subpixel_step has_value */
    float subpixel_step;
    int has_minvar;           /* Config::min_variance has_value */
    float min_variance;       /* UNscaled; match() multiplies by n (cpu.cpp:127) */
    int mode;                 /* 0 LIMITED, 1 FULL */
    int variant;              /* 0 NoDuplicates, 1 Consistency */
    int max_lr_diff;
    int no_dupes;
} bicos_oracle_config;

enum {
    BICOS_ORACLE_NODUPES = 1,     /* BICOSFLAGS_NODUPES     impl/common.hpp:46 */
    BICOS_ORACLE_CONSISTENCY = 2  /* BICOSFLAGS_CONSISTENCY impl/common.hpp:47 */
};

enum {
    BICOS_ORACLE_OUT_INT16 = 0,
    BICOS_ORACLE_OUT_FLOAT32 = 1,
    BICOS_ORACLE_ERR_N = -1,      /* "need at least two images" */
    BICOS_ORACLE_ERR_DEPTH = -2,  /* "bad input depths" */
    BICOS_ORACLE_ERR_BITS = -3    /* std::invalid_argument "input stacks too large" */
};

int bicos_oracle_required_bits(int n, int mode);
int bicos_oracle_desc_words(int n, int mode);

void bicos_oracle_transform(const void* stack, int n, int rows, int cols, int depth,
                            int mode, int words, uint32_t* desc, int nthreads);

void bicos_oracle_search(const uint32_t* desc0, const uint32_t* desc1, int rows, int cols,
                         int words, int flags, int max_lr_diff, int16_t* disp, int nthreads);

void bicos_oracle_agree(int16_t* disp, const void* stack0, const void* stack1, int n,
                        int rows, int cols, int depth, float threshold, int has_minvar,
                        float minvar_scaled, float* corrmap, int nthreads);

void bicos_oracle_agree_subpixel(const int16_t* disp, const void* stack0, const void* stack1,
                                 int n, int rows, int cols, int depth, float threshold,
                                 float step, int has_minvar, float minvar_scaled, float* out,
                                 float* corrmap, int nthreads);

float bicos_oracle_nxcorr(const void* pix0, const void* pix1, int n, int depth, int has_minvar,
                          float minvar_scaled);

/* Full BICOS::match. disp_out must hold rows*cols elements of 4 bytes (int16 results are
 * written as int16 into the first half). corrmap may be NULL. Returns an output kind
 * (BICOS_ORACLE_OUT_*) or a negative error. */
int bicos_oracle_match(const void* stack0, const void* stack1, int n, int rows, int cols,
                       int depth, const bicos_oracle_config* cfg, void* disp_out,
                       float* corrmap, int nthreads);

#ifdef __cplusplus
}
#endif

#endif
