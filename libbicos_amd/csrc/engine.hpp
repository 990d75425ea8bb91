// engine.hpp -- host-side orchestration of the BICOS hot path (internal).
//
// Plays the role of the reference's match_impl (src/impl/cpu.cpp:35-98,
// src/impl/cuda.cu:56-463): transform both stacks, search, optional consistency,
// optional agree / subpixel. All launches are asynchronous on one HIP stream.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <string>

#include "../../include/bicos_c.h"
#include "kernels.hpp"

struct bicos_engine {
    int device = 0;
    int max_lds = 64 * 1024;
    int cus = 256;                     // compute units (workgroup geometry)
    // search kernel tuning (0 = automatic): see bicos_engine_tune
    int tune_variant = 0, tune_R = 0, tune_waves = 0, tune_split = 0;
    hipStream_t own_stream = nullptr;  // used by the host-buffer APIs
    std::mutex lock;                   // serialises host-buffer calls on this engine

    // workspace (grown on demand, never shrunk)
    void* ws = nullptr;
    size_t ws_bytes = 0;
    // host-API staging
    void* stage = nullptr;
    size_t stage_bytes = 0;
};

namespace bicos_impl {

struct Status {
    int code = BICOS_OK;
    std::string msg;
    bool ok() const { return code == BICOS_OK; }
};

void set_error(int code, const std::string& msg);
int fail(int code, const std::string& msg);
int check_hip(hipError_t e, const char* what);

// Reserve `bytes` of engine workspace (device); returns BICOS_OK or an error code.
int reserve(void*& buf, size_t& have, size_t bytes, int device);

int descriptor_words(int n, int mode);

bicos_hip::SearchGeometry geometry(const bicos_engine* e, int rows, int cols, int words);

// Full match on device buffers (validated arguments). corr may be null.
int match_device(bicos_engine* e, const void* s0, const void* s1, int n, int rows, int cols,
                 size_t row_pitch, size_t plane_pitch, int depth, const BicosConfig& cfg,
                 bool has_nxcorr, float threshold, void* disp, void* corr, hipStream_t st);

// Process-wide engine for `device` (created on first use).
bicos_engine* default_engine(int device);

}  // namespace bicos_impl
