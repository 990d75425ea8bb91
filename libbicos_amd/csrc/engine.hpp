// engine.hpp -- host-side orchestration of the BICOS hot path (internal).
//
// Plays the role of the reference's match_impl (src/impl/cpu.cpp:35-98,
// src/impl/cuda.cu:56-463): transform both stacks, search, optional consistency,
// optional agree / subpixel. All launches are asynchronous on one HIP stream.
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bicos_c.h"
#include "kernels.hpp"

namespace bicos_impl {
// Small persistent pool for the host-side copies of the host-buffer pipeline: run(k, f)
// calls f(0..k-1), the caller taking part, and returns when all have finished.
class HostPool {
  public:
    explicit HostPool(int threads);
    ~HostPool();
    int size() const { return (int)workers_.size() + 1; }
    void run(int tasks, const std::function<void(int)>& f);

  private:
    void loop();
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int tasks_ = 0, next_ = 0, active_ = 0;
    unsigned gen_ = 0;
    bool stop_ = false;
};
}  // namespace bicos_impl

struct bicos_engine {
    int device = 0;
    int max_lds = 64 * 1024;           // search row stage budget (>= 2 workgroups per CU)
    int lds_limit = 64 * 1024;         // device limit per workgroup
    int cus = 256;                     // compute units (workgroup geometry)
    // search kernel tuning (0 = automatic): see bicos_engine_tune
    int tune_variant = 0, tune_R = 0, tune_waves = 0, tune_split = 0;
    hipStream_t own_stream = nullptr;  // used by the host-buffer APIs
    std::mutex lock;                   // serialises host-buffer calls on this engine

    // workspace (grown on demand, never shrunk). ws_ready is recorded after every use of
    // ws / stage on the caller's stream and waited on before the next: calls on different
    // streams are ordered, never racing on the shared buffers.
    hipEvent_t ws_ready = nullptr;
    void* ws = nullptr;
    size_t ws_bytes = 0;
    // host-API staging (device): band-major stacks + dense output maps
    void* stage = nullptr;
    size_t stage_bytes = 0;
    // host-buffer pipeline (match_host): copy stream, pinned band slots, band events
    hipStream_t copy_stream = nullptr;
    void* pinned = nullptr;  // K input band slots
    size_t pinned_bytes = 0;
    std::vector<hipEvent_t> events;
    std::unique_ptr<bicos_impl::HostPool> pool;
    // host-staged multi-GPU gather (multi.cpp bicos_match_bands_device): its own pinned
    // buffer and events, grown only (sharing match_host's slots reallocated the
    // pinned memory whenever the two paths alternated)
    void* gather_pinned = nullptr;
    size_t gather_pinned_bytes = 0;
    std::vector<hipEvent_t> gather_events;
    // host-buffer pipeline, maps downloaded band by band on their own stream (so a copy
    // engine other than the uploads' can take them: PCIe is full duplex) into pinned memory,
    // then copied into the caller's buffers by the pool; 2 events per band (matched, landed)
    hipStream_t dl_stream = nullptr;
    // a second upload stream: each band's upload split in two halves (BICOS_HOST_UPLOAD_STREAMS)
    hipStream_t copy_stream2 = nullptr;
    std::vector<hipEvent_t> events2;
    void* pinned_out = nullptr;
    size_t pinned_out_bytes = 0;
    std::vector<hipEvent_t> dl_events;
};

namespace bicos_impl {

struct Status {
    int code = BICOS_OK;
    std::string msg;
    bool ok() const { return code == BICOS_OK; }
};

void set_error(int code, const std::string& msg);
int fail(int code, const std::string& msg);
const char* last_error();  // this thread's last message
int check_hip(hipError_t e, const char* what);

// Reserve `bytes` of engine workspace (device), stream-ordered on `st`: a buffer that
// must grow is freed on `st` after `ready` (every earlier use) and the new one allocated
// there (hipFreeAsync / hipMallocAsync). Returns BICOS_OK or an error code.
int reserve(void*& buf, size_t& have, size_t bytes, int device, hipStream_t st, hipEvent_t ready);

int descriptor_words(int n, int mode);

bicos_hip::SearchGeometry geometry(const bicos_engine* e, int rows, int cols, int words);

// Full match on device buffers (validated arguments). corr may be null. disp_i16: the
// disparity map is int16 even with the NXC stage (no subpixel; bicos_match_device_i16).
// ext_d0 / ext_d1: the two stacks' descriptors (transform output, bicos_desc_pitch rows)
// already computed -- the match then runs from its search on (bicos_search_agree_device).
int match_device(bicos_engine* e, const void* s0, const void* s1, int n, int rows, int cols,
                 size_t row_pitch, size_t plane_pitch, int depth, const BicosConfig& cfg,
                 bool has_nxcorr, float threshold, void* disp, void* corr, hipStream_t st,
                 bool disp_i16 = false, const uint32_t* ext_d0 = nullptr,
                 const uint32_t* ext_d1 = nullptr);

// BICOS_PLAN_* bits of what match_device runs after the transform (bicos_match_plan)
int match_plan(const bicos_engine* e, int n, int rows, int cols, size_t row_pitch,
               size_t plane_pitch, int depth, const BicosConfig& cfg, bool has_nxcorr,
               const void* s0, const void* s1);

// Host buffers in and out (the reference's cv::Mat path, src/impl/cpu.cpp:100-159): the
// stacks are uploaded in row bands through pinned slots on a copy stream while earlier
// bands match on the compute stream; the maps are downloaded into `disp` / `corr` (dense
// rows x cols). p0/p1: n plane pointers each, steps0/steps1: bytes per row of each plane.
// Synchronous.
int match_host(bicos_engine* e, const void* const* p0, const size_t* steps0,
               const void* const* p1, const size_t* steps1, int n, int rows, int cols,
               int depth, const BicosConfig& cfg, bool has_nxcorr, float threshold, void* disp,
               void* corr);

// Process-wide engine for `device` (created on first use).
bicos_engine* default_engine(int device);
bool is_default_engine(const bicos_engine* e);

}  // namespace bicos_impl
