/*
 * bicos_c.h -- C-ABI of libbicos_amd.so, the MI355X (gfx950) BICOS engine.
 *
 * Two layers, both plain C (pointers, sizes, ints; no C++ or torch types):
 *
 * 1. The reference's ctypes ABI, symbol for symbol (drop-in for pybicos_c.so):
 *      BicosConfig / BicosResult          reference src/pybicos_c.cpp:30-53
 *      BICOS_CreateDefaultConfig           reference src/pybicos_c.cpp:92-108
 *      BICOS_FreeConfig                    reference src/pybicos_c.cpp:111-113
 *      BICOS_FreeResult                    reference src/pybicos_c.cpp:116-118
 *      BICOS_Match                         reference src/pybicos_c.cpp:131-200
 *      BICOS_InvalidDisparityFloat/Int16   reference src/pybicos_c.cpp:203-209
 *    Host buffers in, malloc'd host copies out -- exactly the reference contract,
 *    with three documented fixes:
 *      - BicosConfig ALWAYS carries `precision` (the reference's Python wrapper,
 *        pybicos/__init__.py:41-51, always lays it out; the reference's CPU build
 *        omitted it and silently shifted the struct);
 *      - BICOS_FreeResult frees the data buffers too (the reference leaked them);
 *      - every exception is caught at the boundary (NULL result), not only
 *        BICOS::Exception; bicos_last_error() says why.
 *
 * 2. The device-resident hot path (bicos_hip_*): device pointers to planar image
 *    stacks already in HBM, results written to caller-provided device buffers,
 *    asynchronous on the caller's HIP stream. This is the entry point the
 *    reference's CUDA build exposes through BICOS::match(GpuMat...) with a
 *    cv::cuda::Stream (reference include/match.hpp:31-41, src/impl/cuda.cu:465-524),
 *    restated without OpenCV types.
 *
 * Error convention: int-returning functions return BICOS_OK (0) or a negative
 * BICOS_E_* code; bicos_last_error() returns a thread-local message.
 */
#ifndef BICOS_C_H
#define BICOS_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* OpenCV type codes used across the ABI (CV_MAKETYPE(depth, 1)) */
#define BICOS_CV_8U 0
#define BICOS_CV_16U 2
#define BICOS_CV_16S 3
#define BICOS_CV_32F 5
#define BICOS_CV_64F 6

/* reference src/pybicos_c.cpp:30-41 (with `precision` unconditionally present) */
typedef struct {
    float nxcorr_threshold; /* < 0: keep the default 0.5 (reference :59-61) */
    float subpixel_step;    /* < 0: no subpixel refinement */
    float min_variance;     /* < 0: no minimum variance */
    int mode;               /* 0 = LIMITED, 1 = FULL */
    int precision;          /* 0 = SINGLE, 1 = DOUBLE */
    int variant_type;       /* 0 = NoDuplicates, 1 = Consistency */
    int max_lr_diff;        /* Consistency only */
    int no_dupes;           /* Consistency only */
} BicosConfig;

/* reference src/pybicos_c.cpp:44-53 */
typedef struct {
    void* disparity_data;
    int disparity_rows;
    int disparity_cols;
    int disparity_type;
    void* corrmap_data;
    int corrmap_rows;
    int corrmap_cols;
    int corrmap_type;
} BicosResult;

BicosConfig* BICOS_CreateDefaultConfig(void);
void BICOS_FreeConfig(BicosConfig* config);
void BICOS_FreeResult(BicosResult* result);
BicosResult* BICOS_Match(void** stack0_data, int* stack0_rows, int* stack0_cols, int* stack0_types,
                         int stack0_size, void** stack1_data, int* stack1_rows, int* stack1_cols,
                         int* stack1_types, int stack1_size, BicosConfig* config);
float BICOS_InvalidDisparityFloat(void);
int16_t BICOS_InvalidDisparityInt16(void);

/* ------------------------------------------------------------------ errors */
enum {
    BICOS_OK = 0,
    BICOS_E_ARG = -1,       /* invalid argument (BICOS::Exception in the reference) */
    BICOS_E_BITS = -2,      /* stacks need > 256 descriptor bits (std::invalid_argument) */
    BICOS_E_HIP = -3,       /* HIP runtime error */
    BICOS_E_INTERNAL = -4
};
const char* bicos_last_error(void);

/* --------------------------------------------------- device-resident API */

/* Opaque per-device engine: owns a workspace (descriptor buffers, temporaries)
 * that grows on demand (stream-ordered: hipFreeAsync / hipMallocAsync on the calling
 * stream, never a device-wide synchronisation) and is reused across calls. Calls on one
 * handle from several host threads are serialised by the engine's lock; the GPU work of
 * calls on different streams is ordered through the engine's workspace event. */
typedef struct bicos_engine bicos_engine;

int bicos_engine_create(int device, bicos_engine** out);
/* The process-wide engine of `device` that BICOS_Match, bicos_match_host(NULL, ...) and
 * BICOS::match use (created on first use; bicos_engine_destroy ignores it). NULL on error. */
bicos_engine* bicos_engine_default(int device);
void bicos_engine_destroy(bicos_engine* e);

/* Search-kernel tuning for this engine (0 = automatic for each argument):
 *   variant        16 = the VALU search (packed 16-bit keys)
 *   col0_per_lane  left pixels held in registers per lane (2|4)
 *   waves          waves per workgroup (1..8)
 *   split          waves that share one col0 group and split its col1 scan (1|2|4|8)
 * Matrix-core search (search_mx.hip, the default): variant 64 (automatic keys), 65 (one FP4
 * product per pair + xor keys; rows <= 16384), 66 (two products: first / last minimum), 67
 * (xor keys for first-minimum searches too, instead of the float keys that carry the column
 * in a free K half);
 * col0_per_lane = 32-column tiles per wave (2|4|8; 8 falls back to 4 where the registers do
 * not fit), waves 1..8, split = LDS stage KiB (0 = 64).
 * Results are identical for every setting; only speed changes. */
int bicos_engine_tune(bicos_engine* e, int variant, int col0_per_lane, int waves, int split);

/* Descriptor width in 32-bit words for n images in `mode` (reference dispatch
 * src/impl/cpu.cpp:122-156); BICOS_E_BITS when more than 256 bits are needed. */
int bicos_descriptor_words(int n, int mode);

/* Output element type BICOS_Match / bicos_match_device produce for a config:
 * BICOS_CV_16S without a correlation threshold, else BICOS_CV_32F
 * (BICOS_CV_64F corrmap for precision DOUBLE). */
int bicos_output_type(const BicosConfig* cfg, int has_nxcorr);

/*
 * Full match on device-resident planar stacks.
 *   stack0/stack1 : n planes each; element (t, y, x) at
 *                   base[t*plane_pitch + y*row_pitch + x], u8 (depth 1) or u16 (depth 2)
 *   has_nxcorr    : 0 disables the NXC stage (Config::nxcorr_threshold = nullopt, only
 *                   reachable from C++ in the reference); disparity is then int16
 *   disparity     : device, rows*cols dense, int16 or float32 per bicos_output_type
 *   corrmap       : device, rows*cols dense float32 (float64 for DOUBLE), or NULL
 *   stream        : hipStream_t (NULL = default stream); the call only enqueues work
 */
int bicos_match_device(bicos_engine* e, const void* stack0, const void* stack1, int n, int rows,
                       int cols, size_t row_pitch, size_t plane_pitch, int depth,
                       const BicosConfig* cfg, int has_nxcorr, void* disparity, void* corrmap,
                       void* stream);

/*
 * bicos_match_device with the disparity map always int16, also with the NXC stage: the
 * integer disparity, -32768 where invalid or below the threshold, so that
 * (float)disparity is exactly the float32 map bicos_match_device writes (the reference's
 * float map is the int16 one converted, src/impl/cpu.cpp:77-95). Half the bytes of the
 * float map -- what a row band ships to the gathering GPU (bench.py). A subpixel config
 * is rejected (BICOS_E_ARG): its disparities are not integers. No reference counterpart.
 */
int bicos_match_device_i16(bicos_engine* e, const void* stack0, const void* stack1, int n,
                           int rows, int cols, size_t row_pitch, size_t plane_pitch, int depth,
                           const BicosConfig* cfg, int has_nxcorr, void* disparity, void* corrmap,
                           void* stream);

/*
 * Full match on host buffers (the reference's cv::Mat path; what BICOS_Match and
 * pybicos.match run). Synchronous.
 *   e             : engine, or NULL for the current device's default engine
 *   stack0/stack1 : n host image pointers each (any addresses), rows x cols, `step` bytes
 *                   per row (0 = dense), u8 (depth 1) or u16 (depth 2)
 *   disparity     : host, rows*cols dense, int16 or float32 per bicos_output_type
 *   corrmap       : host, rows*cols dense float32 (float64 for DOUBLE), or NULL
 * The stacks are uploaded in row bands through pinned staging on a copy stream while the
 * bands already uploaded are matched; the maps are written straight into the buffers.
 */
int bicos_match_host(bicos_engine* e, const void* const* stack0, const void* const* stack1, int n,
                     int rows, int cols, size_t step, int depth, const BicosConfig* cfg,
                     int has_nxcorr, void* disparity, void* corrmap);

/* ------------------------------------------------ single-process multi-GPU */
/* One frame matched on several GPUs from one process (the reference has
 * no multi-GPU API -- these extend bicos_match_host / bicos_match_device, whose conventions
 * they keep). The frame's rows are split into contiguous bands, band b on devices[b] with
 * that device's default engine. Every stage of the match is row-local, so the maps are
 * byte-identical to the one-GPU call. devices may repeat (bands on one GPU then run one
 * after another on its engine). Both calls are synchronous. */

/* Host buffers, bicos_match_host's arguments: the rows are split into min(ndev, rows)
 * bands whose heights differ by at most one (the first rows % ndev bands get the extra
 * row); one host thread per band runs the banded upload -> match -> download pipeline of
 * its GPU over that GPU's own PCIe link and writes its rows of the maps straight into
 * `disparity` / `corrmap`. */
int bicos_match_host_multi(const int* devices, int ndev, const void* const* stack0,
                           const void* const* stack1, int n, int rows, int cols, size_t step,
                           int depth, const BicosConfig* cfg, int has_nxcorr, void* disparity,
                           void* corrmap);

/* Device-resident bands: band b (band_rows[b] rows, in frame order) lives on devices[b] as
 * planar stacks stack0[b] / stack1[b] with row_pitch[b] / plane_pitch[b] (elements, as in
 * bicos_match_device). Each GPU matches its band; the maps are gathered into `disparity` /
 * `corrmap` on devices[0] (dense, sum(band_rows) x cols; corrmap may be NULL) by peer
 * copies over xGMI -- band 0 is written in place. */
int bicos_match_bands_device(const int* devices, int ndev, const void* const* stack0,
                             const void* const* stack1, const int* band_rows,
                             const size_t* row_pitch, const size_t* plane_pitch, int n, int cols,
                             int depth, const BicosConfig* cfg, int has_nxcorr, void* disparity,
                             void* corrmap);

/* Stage entry points (tests, benchmarks, custom pipelines). Same conventions.
 * desc buffers: rows x desc_pitch uint32 with desc_pitch = bicos_desc_pitch(cols, words). */
size_t bicos_desc_pitch(int cols, int words);
int bicos_transform_device(const void* stack, int n, int rows, int cols, size_t row_pitch,
                           size_t plane_pitch, int depth, int mode, int words, uint32_t* desc,
                           void* stream);
/* flags: 1 = NODUPES, 2 = CONSISTENCY (reference impl/common.hpp:46-47). Consistency needs
 * the engine's workspace; out is int16 rows x cols (dense).
 * flags bits 16-24 (optional): B = (flags >> 16) & 0x1FF, the number of low descriptor bits
 * that may be set (0 = all). The caller promises bits B..32*words-1 are zero in both
 * descriptor sets (true of transform output with B >= the transform's bit count: LIMITED
 * 4n-6, FULL n^2-2n+3); the matrix-core search then skips the 64-bit K-steps above B
 * (256-bit descriptors with B <= 192: 3 steps instead of 4). Results are unchanged.
 * 256-bit descriptors (words = 8): bit 255 is ignored (masked on both sides). Every
 * descriptor the transform produces leaves it zero -- LIMITED uses at most 4*65-6 = 254
 * bits, FULL at most 16*16-2*16+3 = 227 -- so results on transform output are exact; a
 * caller passing hand-made descriptors must keep bit 255 clear. */
int bicos_search_device(bicos_engine* e, const uint32_t* desc0, const uint32_t* desc1, int rows,
                        int cols, int words, int flags, int max_lr_diff, int16_t* out,
                        void* stream);
/* agree: raw int16 disparity -> float32 disparity (+ corrmap); minvar already x n */
int bicos_agree_device(const int16_t* raw, const void* stack0, const void* stack1, int n, int rows,
                       int cols, size_t row_pitch, size_t plane_pitch, int depth, float threshold,
                       int has_minvar, float minvar_scaled, float* out, float* corrmap,
                       void* stream);
int bicos_subpixel_device(const int16_t* raw, const void* stack0, const void* stack1, int n,
                          int rows, int cols, size_t row_pitch, size_t plane_pitch, int depth,
                          float threshold, float step, int has_minvar, float minvar_scaled,
                          float* out, float* corrmap, void* stream);
/* agree (step <= 0) or subpixel (step > 0) in either precision: precision 1 = the CUDA
 * build's Precision::DOUBLE NXC (corrmap is then double*); the reference kernel-bench shapes
 * (bench/cuda.cu:99-180) time these with double precision. */
int bicos_agree_stage_device(const int16_t* raw, const void* stack0, const void* stack1, int n,
                             int rows, int cols, size_t row_pitch, size_t plane_pitch, int depth,
                             float threshold, float step, int has_minvar, float minvar_scaled,
                             int precision, float* out, void* corrmap, void* stream);

/* What bicos_match_device runs for a shape and config past the descriptor transform
 * (tests, benchmarks): a mask of BICOS_PLAN_* bits, or a negative BICOS_E_* code for an
 * invalid configuration. stack0 / stack1 are only inspected for their alignment. No
 * reference counterpart (its kernels are fixed per build). */
#define BICOS_PLAN_MATRIX_CORES 1           /* the FP4 MFMA search (search_mx.hip) */
#define BICOS_PLAN_PACKED_KEYS 2            /* its packed-key form (search_pk_kernel) */
#define BICOS_PLAN_AGREE_IN_SEARCH 4        /* the NXC agree inside the search launch */
#define BICOS_PLAN_REVERSE_COMPACTED 8      /* Consistency: reverse search over kept col1 */
#define BICOS_PLAN_CONSISTENCY_IN_AGREE 16  /* Consistency: left-right check in the agree */
#define BICOS_PLAN_DENSE_ROWS 32            /* ... rows kept >= 7/8 skip the entry prologue */
#define BICOS_PLAN_CONSISTENCY_ONE_PASS 64  /* Consistency: both searches + the check, one launch */
int bicos_match_plan(bicos_engine* e, const void* stack0, const void* stack1, int n, int rows,
                     int cols, size_t row_pitch, size_t plane_pitch, int depth,
                     const BicosConfig* cfg, int has_nxcorr);

/* bicos_match_device from its search on: desc0 / desc1 are the two stacks' descriptors as
 * bicos_transform_device writes them (rows x bicos_desc_pitch(cols, words) uint32, words =
 * bicos_descriptor_words(n, cfg->mode)); the stacks are still read by the agree / subpixel
 * stage. Exactly the launches the match issues after its transform (bicos_match_plan), so
 * benchmarks can time them in isolation; same outputs as bicos_match_device. */
int bicos_search_agree_device(bicos_engine* e, const uint32_t* desc0, const uint32_t* desc1,
                              const void* stack0, const void* stack1, int n, int rows, int cols,
                              size_t row_pitch, size_t plane_pitch, int depth,
                              const BicosConfig* cfg, int has_nxcorr, void* disparity,
                              void* corrmap, void* stream);

/* Build identification (arch, flags) for reports. */
const char* bicos_build_info(void);

#ifdef __cplusplus
}
#endif

#endif /* BICOS_C_H */
