// engine.cpp -- host orchestration of the gfx950 BICOS hot path + the C++ API.
//
//   bicos_impl::match_device   <- reference match_impl (src/impl/cpu.cpp:35-98)
//   BICOS::match               <- reference BICOS::match (src/lib.cpp:31-49) and the
//                                 backend entry impl::cpu::match (src/impl/cpu.cpp:100-159)
#include "engine.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <vector>

#include "../../include/bicos/common.hpp"
#include "../../include/bicos/match.hpp"
#include "../../include/bicos/hip.hpp"

namespace bicos_impl {

namespace {
thread_local std::string g_last_error;

constexpr size_t ALIGN = 256;
size_t align_up(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }
}  // namespace

void set_error(int code, const std::string& msg) {
    (void)code;
    g_last_error = msg;
}

int fail(int code, const std::string& msg) {
    set_error(code, msg);
    return code;
}

int check_hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return BICOS_OK;
    std::ostringstream os;
    os << what << ": " << hipGetErrorName(e) << " (" << hipGetErrorString(e) << ")";
    return fail(BICOS_E_HIP, os.str());
}

const char* last_error() { return g_last_error.c_str(); }

int reserve(void*& buf, size_t& have, size_t bytes, int device, hipStream_t st,
            hipEvent_t ready) {
    if (bytes <= have && buf) return BICOS_OK;
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    int rc = BICOS_OK;
    if (buf) {
        // Stream-ordered: every earlier use of the old buffer, on any stream, is ordered
        // before `ready` (recorded after each use), so `st` waits for it and frees the old
        // buffer in its own order -- no device-wide synchronisation, nothing else stalls.
        rc = check_hip(hipStreamWaitEvent(st, ready, 0), "hipStreamWaitEvent");
        if (!rc) rc = check_hip(hipFreeAsync(buf, st), "hipFreeAsync(workspace)");
        buf = nullptr;
        have = 0;
    }
    const size_t want = bytes + bytes / 8;  // headroom for slightly larger calls
    if (!rc) rc = check_hip(hipMallocAsync(&buf, want, st), "hipMallocAsync(workspace)");
    if (cur != device) (void)hipSetDevice(cur);
    if (rc != BICOS_OK) {
        buf = nullptr;
        return rc;
    }
    have = want;
    return BICOS_OK;
}

// reference src/impl/cpu.cpp:122-156
int descriptor_words(int n, int mode) {
    const long bits = mode ? (long)n * n - 2L * n + 3 : 4L * n - 7;
    if (bits <= 32) return 1;
    if (bits <= 64) return 2;
    if (bits <= 128) return 4;
    if (bits <= 256) return 8;
    return BICOS_E_BITS;
}

bicos_hip::SearchGeometry geometry(const bicos_engine* e, int rows, int cols, int words) {
    int max_lds = e ? e->max_lds : 64 * 1024;
    // Row stage budget per workgroup (BICOS_SEARCH_STAGE_KIB, default 40; 0 = whole rows up
    // to 64 KiB): wider rows are split into equal chunks under it, so 4 workgroups (8 waves
    // per SIMD) stay resident per CU. Measured: 3840-column rows (cfg5) search -2.6 %,
    // 256-bit 2048-column rows -1.3 %; rows that fit (cfg2: 32 KiB) are unchanged.
    static const int stage_kib = [] {
        const char* v = std::getenv("BICOS_SEARCH_STAGE_KIB");
        return v ? std::atoi(v) : 40;
    }();
    if (stage_kib > 0) {
        const int budget = stage_kib * 1024;
        const int bytes = cols * words * 4;
        if (bytes > budget) {
            const int chunks = (bytes + budget - 1) / budget;
            const int chunk = (cols + chunks - 1) / chunks;
            max_lds = std::min(max_lds, chunk * words * 4);
        }
    }
    // (an engine tuned for the matrix-core search runs VALU kernels untuned)
    if (!e || e->tune_variant >= 64) return bicos_hip::search_geometry(rows, cols, words, max_lds);
    return bicos_hip::search_geometry(rows, cols, words, max_lds, e->tune_variant, e->tune_R,
                                      e->tune_waves, e->tune_split, e->cus);
}

// The agree inside the search launch for the shape search_mx_agree_fusable accepts
// (BICOS_FUSE_AGREE=0: the separate agree launch; read once)
static bool fuse_agree() {
    static const bool on = [] {
        const char* v = std::getenv("BICOS_FUSE_AGREE");
        return !(v && !std::strcmp(v, "0"));
    }();
    return on;
}
// Consistency's left-right check inside the agree launch (kernels.hip agree_lds_kernel CONS;
// BICOS_FUSE_CONS=0: consistency_kernel + the agree; read once)
static bool fuse_consistency() {
    static const bool on = [] {
        const char* v = std::getenv("BICOS_FUSE_CONS");
        return !(v && !std::strcmp(v, "0"));
    }();
    return on;
}

// Search implementation: the matrix-core search (search_mx.hip) unless the engine is tuned
// to the VALU search (bicos_engine_tune variant 16) or BICOS_SEARCH=valu;
// BICOS_SEARCH=mx forces it. Results are identical either way.
bool use_mx(const bicos_engine* e) {
    static const int env = [] {
        const char* v = std::getenv("BICOS_SEARCH");
        if (!v) return 0;
        if (!std::strcmp(v, "valu")) return 1;
        if (!std::strcmp(v, "mx")) return 2;
        return 0;
    }();
    if (e && e->tune_variant >= 64) return true;
    if (e && e->tune_variant != 0) return false;
    return env != 1;
}

// Highest descriptor bit the transform writes + 1 (an upper bound: LIMITED writes 4n-6 bits
// for n >= 4, 7 for n = 3 and 4 for n = 2 -- the closing four comparisons alone,
// descriptor_transform.hpp:62-68 --, FULL n^2-2n+3; descriptor_transform.hpp:31-123). The
// search multiplies only the 64-bit K-steps that hold them.
int used_bits(int n, int mode) { return mode ? n * n - 2 * n + 3 : std::max(4 * n - 5, 4); }

bicos_hip::MxGeometry mx_geometry(const bicos_engine* e, int rows, int cols, int words,
                                  int bits = 0) {
    const bool tuned = e && e->tune_variant >= 64;
    // tuned: split = LDS stage KiB (0 = 64)
    const int lds = tuned && e->tune_split > 0 ? e->tune_split * 1024 : 64 * 1024;
    return bicos_hip::search_mx_geometry(rows, cols, words, lds, tuned ? e->tune_R : 0,
                                         tuned ? e->tune_waves : 0, e ? e->cus : 256,
                                         tuned ? e->tune_variant - 64 : 0, bits);
}

// Number of x the reference's subpixel loop visits: for (float x = -1.f; x <= 1.f; x += step)
// (agree.hpp:122 / agree.cuh:213), accumulated in float exactly as there. 0 when the loop
// would exceed MAX_SUBPIXEL_STEPS (or never end: x + step == x), which the reference would
// run for hours on a CPU and which on a GPU is a hung device; such steps are rejected.
constexpr int MAX_SUBPIXEL_STEPS = 65536;
int subpixel_steps(float step) {
    int count = 0;
    for (float x = -1.f; x <= 1.f; x += step)
        if (++count > MAX_SUBPIXEL_STEPS) return 0;
    return count;
}

static int required_bits(int n, int mode) { return mode ? n * n - 2 * n + 3 : 4 * n - 7; }

// Consistency's reverse search (reference bicos.hpp:94-106, bicos.cuh:110-135): rev[col1] is
// read only for the col1 a valid forward match chose, so the matrix-core search runs only
// over those -- per row the distinct valid fwd[col0] in ascending order, which each
// workgroup of the compacted search finds itself (search_mx.hip list_prologue); rev
// elsewhere is left unwritten and never read. Periodic inputs whose forward search keeps
// nothing skip the reverse pass almost entirely. BICOS_REV_FULL=1 (A/B) and the VALU search
// run the full reverse pass. `run(keep)` launches the reverse search, keep = nullptr: full.
static bool reverse_compacted(bool mx) {
    static const bool full = [] {
        const char* v = std::getenv("BICOS_REV_FULL");
        return v && std::atoi(v) != 0;
    }();
    return mx && !full;
}

// Consistency's dense-row fast path (SearchArgs.row_valid, search_mx.hip dense_row): the
// forward search counts its valid col0 per 32-column tile and the compacted reverse search
// skips its entry prologue on rows that kept >= 7/8 of them. BICOS_DENSE_ROWS=0: off (A/B).
static bool dense_rows() {
    static const bool on = [] {
        const char* v = std::getenv("BICOS_DENSE_ROWS");
        return !(v && !std::strcmp(v, "0"));
    }();
    return on;
}
// Consistency without NoDuplicates in one launch where the descriptors allow it (search_mx.hip
// search_lr_kernel: the forward and reverse searches share their matrix products, the check
// runs in the same workgroup). BICOS_LR_ONE_PASS=0: the two searches + the check (A/B; read
// per call, so one process can compare the two forms).
static bool lr_one_pass() {
    const char* v = std::getenv("BICOS_LR_ONE_PASS");
    return !(v && !std::strcmp(v, "0"));
}
// Descriptor bits the transform writes, exactly (descriptor_transform.hpp:31-123; used_bits
// is an upper bound): LIMITED 4n-6 for n >= 4 (7 for n = 3, 4 for n = 2), FULL n^2-2n+3
static int written_bits(int n, int mode) {
    if (mode) return n * n - 2 * n + 3;
    return n >= 4 ? 4 * n - 6 : (n == 3 ? 7 : 4);
}
// bytes per row of the per-tile valid counts
static size_t valid_pitch(int cols) { return ((size_t)(cols + 31) / 32 + 15) / 16 * 16; }

// Bytes the kernels may address from a stack base; the kernels use 32-bit buffer offsets.
static int stack_span(int n, int rows, int cols, size_t row_pitch, size_t plane_pitch, int depth,
                      uint32_t* out) {
    if (rows <= 0 || cols <= 0) {
        *out = 0;
        return BICOS_OK;
    }
    const unsigned long long span =
        ((unsigned long long)(n - 1) * plane_pitch + (unsigned long long)(rows - 1) * row_pitch +
         (unsigned long long)cols) * (unsigned long long)depth;
    if (span > 0xFFFFFFFFull) return fail(BICOS_E_ARG, "image stack spans more than 4 GiB");
    *out = (uint32_t)span;
    return BICOS_OK;
}

// What match_device runs for a shape and config (bicos_match_plan's bits, bicos_c.h): the
// kernels after the transform. Valid configurations only (match_device validates first).
int match_plan(const bicos_engine* e, int n, int rows, int cols, size_t row_pitch,
               size_t plane_pitch, int depth, const BicosConfig& cfg, bool has_nxcorr,
               const void* s0, const void* s1) {
    const int mode = cfg.mode == 0 ? 0 : 1;
    const int words = descriptor_words(n, mode);
    if (words < 0 || rows <= 0 || cols <= 0) return 0;
    const bool consistency = cfg.variant_type != 0;
    const bool nodupes = consistency ? cfg.no_dupes != 0 : true;
    const bool has_step = has_nxcorr && cfg.subpixel_step >= 0;
    const bool dbl = cfg.precision != 0;
    const bool mx = use_mx(e);
    // the LDS-staged agree kernels read the left planes with dword loads
    const bool aligned4 = ((row_pitch * depth | plane_pitch * depth) & 3) == 0 &&
                          (((uintptr_t)s0 | (uintptr_t)s1) & 3) == 0;
    int plan = 0;
    if (mx) {
        plan |= BICOS_PLAN_MATRIX_CORES;
        const bicos_hip::MxGeometry g = mx_geometry(e, rows, cols, words, used_bits(n, mode));
        if (g.pk && nodupes) plan |= BICOS_PLAN_PACKED_KEYS;
        if (!consistency && has_nxcorr && !has_step && aligned4 && fuse_agree() &&
            bicos_hip::search_mx_agree_fusable(g, words, true, cols, n, depth, dbl))
            plan |= BICOS_PLAN_AGREE_IN_SEARCH;
    }
    if (consistency && mx && !nodupes && lr_one_pass() &&
        bicos_hip::search_lr_eligible(words, written_bits(n, mode), cols))
        return plan | BICOS_PLAN_CONSISTENCY_ONE_PASS;
    if (consistency) {
        if (reverse_compacted(mx)) {
            plan |= BICOS_PLAN_REVERSE_COMPACTED;
            if (dense_rows()) plan |= BICOS_PLAN_DENSE_ROWS;
        }
        if (has_nxcorr && !has_step && aligned4 && n <= 65 && fuse_consistency())
            plan |= BICOS_PLAN_CONSISTENCY_IN_AGREE;
    }
    return plan;
}

int match_device(bicos_engine* e, const void* s0, const void* s1, int n, int rows, int cols,
                 size_t row_pitch, size_t plane_pitch, int depth, const BicosConfig& cfg,
                 bool has_nxcorr, float threshold, void* disp, void* corr, hipStream_t st,
                 bool disp_i16, const uint32_t* ext_d0, const uint32_t* ext_d1) {
    if (!e) return fail(BICOS_E_ARG, "null engine");
    if (n < 2) return fail(BICOS_E_ARG, "need at least two images");
    if (depth != 1 && depth != 2)
        return fail(BICOS_E_ARG, "bad input depths, only CV_8UC1 and CV_16UC1 are supported");
    if (rows < 0 || cols < 0) return fail(BICOS_E_ARG, "negative image size");
    if (cols > 32767)
        return fail(BICOS_E_ARG, "image width exceeds the int16 disparity range (32767)");
    const int mode = cfg.mode == 0 ? 0 : 1;
    const int words = descriptor_words(n, mode);
    if (words < 0) {
        std::ostringstream os;
        os << "input stacks too large, would require " << required_bits(n, mode) << " bits";
        return fail(BICOS_E_BITS, os.str());
    }
    const bool has_step = has_nxcorr && cfg.subpixel_step >= 0;
    if (has_step && !(cfg.subpixel_step > 0 && std::isfinite(cfg.subpixel_step)))
        return fail(BICOS_E_ARG, "subpixel_step must be a positive finite number");
    const int nsteps = has_step ? subpixel_steps(cfg.subpixel_step) : 0;
    if (has_step && !nsteps)
        return fail(BICOS_E_ARG, "subpixel_step too small (more than 65536 interpolation steps)");
    if (disp_i16 && has_step)
        return fail(BICOS_E_ARG, "an int16 disparity map cannot hold subpixel disparities");
    if (rows == 0 || cols == 0) return BICOS_OK;
    if (!s0 || !s1 || !disp) return fail(BICOS_E_ARG, "null buffer");
    if (row_pitch < (size_t)cols || plane_pitch < (size_t)rows * row_pitch)
        return fail(BICOS_E_ARG, "row/plane pitch smaller than the image");
    uint32_t span = 0;
    if (int rc0 = stack_span(n, rows, cols, row_pitch, plane_pitch, depth, &span)) return rc0;

    const bool consistency = cfg.variant_type != 0;
    const bool nodupes = consistency ? cfg.no_dupes != 0 : true;
    const bool dbl = cfg.precision != 0;

    const bool mx = use_mx(e);

    const int plan = match_plan(e, n, rows, cols, row_pitch, plane_pitch, depth, cfg, has_nxcorr,
                                s0, s1);
    // workspace: desc0 | desc1 | raw int16 | fwd | rev (Consistency); the descriptors are the
    // caller's when given (bicos_search_agree_device: the match past its transform)
    const size_t dpitch = bicos_desc_pitch(cols, words);
    const bool ext = ext_d0 != nullptr;
    if (ext != (ext_d1 != nullptr)) return fail(BICOS_E_ARG, "need both descriptor buffers");
    const size_t desc_bytes = ext ? 0 : align_up((size_t)rows * dpitch * 4);
    const size_t map16 = align_up((size_t)rows * cols * 2);
    const size_t vpitch = valid_pitch(cols);
    const size_t vbytes = (plan & BICOS_PLAN_DENSE_ROWS) ? align_up((size_t)rows * vpitch) : 0;
    const bool two_maps = consistency && !(plan & BICOS_PLAN_CONSISTENCY_ONE_PASS);
    size_t need = 2 * desc_bytes + (has_nxcorr ? map16 : 0) + (two_maps ? 2 * map16 : 0) + vbytes;
    int rc = reserve(e->ws, e->ws_bytes, need, e->device, st, e->ws_ready);
    if (rc) return rc;
    // order against earlier users of ws / stage on other streams; mark our use on exit
    rc = check_hip(hipStreamWaitEvent(st, e->ws_ready, 0), "hipStreamWaitEvent");
    if (rc) return rc;
    struct MarkUse {
        hipEvent_t ev;
        hipStream_t st;
        ~MarkUse() { (void)hipEventRecord(ev, st); }
    } mark{e->ws_ready, st};
    char* p = (char*)e->ws;
    const uint32_t* d0 = ext ? ext_d0 : (const uint32_t*)p;
    p += desc_bytes;
    const uint32_t* d1 = ext ? ext_d1 : (const uint32_t*)p;
    p += desc_bytes;
    int16_t* raw = has_nxcorr ? (int16_t*)p : (int16_t*)disp;
    if (has_nxcorr) p += map16;
    int16_t* fwd = two_maps ? (int16_t*)p : nullptr;
    int16_t* rev = two_maps ? (int16_t*)(p + map16) : nullptr;
    uint8_t* valid = vbytes ? (uint8_t*)(p + 2 * map16) : nullptr;  // dense-row fast path

    // 1. descriptor_transform, both stacks in one launch (cpu.cpp:50-59)
    if (!ext) {
        bicos_hip::TransformArgs ta{s0, s1, (uint32_t*)d0, (uint32_t*)d1, n, rows, cols,
                                    row_pitch, plane_pitch, dpitch, 0, span};
        rc = check_hip(bicos_hip::launch_transform(ta, depth, mode, words, st), "transform launch");
        if (rc) return rc;
    }

    // 2. bicos search (cpu.cpp:68-75): NoDuplicates in one search; Consistency as the
    // forward and the reverse search (the same search with the stacks swapped, bicos.hpp:96)
    // over only the col1 the forward search kept (reverse_search), then the left-right check
    auto search = [&](const uint32_t* a0, const uint32_t* a1, int16_t* out, int out_mode,
                      bool nd, const char* what, const int16_t* keep = nullptr,
                      uint8_t* row_valid = nullptr) {
        bicos_hip::SearchArgs sa{a0, a1, out, rows, cols, dpitch, (size_t)cols, out_mode, 0, 0, 0};
        sa.keep = keep;
        sa.keep_pitch = (size_t)cols;
        sa.row_valid = row_valid;
        sa.valid_pitch = vpitch;
        if (mx)
            return check_hip(bicos_hip::launch_search_mx(
                                 sa, mx_geometry(e, rows, cols, words, used_bits(n, mode)), words, nd, st),
                             what);
        return check_hip(bicos_hip::launch_search(sa, geometry(e, rows, cols, words), words, nd, st),
                         what);
    };
    // 3. agree / agree_subpixel (cpu.cpp:77-95)
    bicos_hip::AgreeArgs aa{};
    aa.raw = raw;
    aa.raw_pitch = (size_t)cols;
    aa.stack0 = s0;
    aa.stack1 = s1;
    aa.n = n;
    aa.rows = rows;
    aa.cols = cols;
    aa.row_pitch = row_pitch;
    aa.plane_pitch = plane_pitch;
    aa.threshold = threshold;
    aa.step = has_step ? cfg.subpixel_step : 0.f;
    aa.nsteps = nsteps;
    aa.has_minvar = cfg.min_variance >= 0;
    aa.minvar = aa.has_minvar ? cfg.min_variance * (float)n : 0.f;  // cpu.cpp:127
    aa.out = disp;
    aa.out_f32 = disp_i16 ? 0 : 1;
    aa.corrmap = corr;
    aa.stack_bytes = span;

    // the headline shape runs the agree inside the search's workgroups (one launch,
    // search_mx.hip fused_agree; BICOS_FUSE_AGREE=0 keeps the two launches)
    if (plan & BICOS_PLAN_AGREE_IN_SEARCH) {
        const bicos_hip::MxGeometry g = mx_geometry(e, rows, cols, words, used_bits(n, mode));
        bicos_hip::SearchArgs sa{d0, d1, raw, rows, cols, dpitch, (size_t)cols, 0, 0, 0, 0};
        return check_hip(bicos_hip::launch_search_mx_agree(sa, aa, g, st), "search + agree launch");
    }

    if (plan & BICOS_PLAN_CONSISTENCY_ONE_PASS) {
        bicos_hip::SearchArgs sa{d0, d1, raw, rows, cols, dpitch, (size_t)cols, 0, 0, 0, 0};
        rc = check_hip(bicos_hip::launch_search_lr(sa, words, written_bits(n, mode), cfg.max_lr_diff, st),
                       "consistency search launch");
        if (rc) return rc;
    } else if (!consistency) {
        rc = search(d0, d1, raw, 0, true, "search launch");
        if (rc) return rc;
    } else {
        rc = search(d0, d1, fwd, 1, nodupes, "search launch", nullptr, valid);
        if (!rc)
            rc = search(d1, d0, rev, 1, nodupes, "reverse search launch",
                        (plan & BICOS_PLAN_REVERSE_COMPACTED) ? fwd : nullptr, valid);
        if (rc) return rc;
        if (plan & BICOS_PLAN_CONSISTENCY_IN_AGREE) {
            // the left-right check runs inside the agree (kernels.hip agree_lds_kernel CONS)
            aa.fwd = fwd;
            aa.rev = rev;
            aa.max_lr_diff = cfg.max_lr_diff;
            return check_hip(bicos_hip::launch_agree(aa, depth, dbl, st), "consistency + agree launch");
        }
        bicos_hip::ConsistencyArgs ca{fwd, rev, raw, rows, cols, (size_t)cols, cfg.max_lr_diff};
        rc = check_hip(bicos_hip::launch_consistency(ca, st), "consistency launch");
        if (rc) return rc;
    }
    if (!has_nxcorr) return BICOS_OK;

    if (has_step)
        rc = check_hip(bicos_hip::launch_subpixel(aa, depth, dbl, st), "subpixel launch");
    else
        rc = check_hip(bicos_hip::launch_agree(aa, depth, dbl, st), "agree launch");
    return rc;
}

// ------------------------------------------------------- host-buffer pipeline

HostPool::HostPool(int threads) {
    for (int i = 1; i < threads; ++i) workers_.emplace_back([this] { loop(); });
}

HostPool::~HostPool() {
    {
        std::lock_guard<std::mutex> g(m_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
}

void HostPool::loop() {
    unsigned seen = 0;
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        ++active_;
        while (next_ < tasks_) {
            const int i = next_++;
            const std::function<void(int)>* f = job_;
            lk.unlock();
            (*f)(i);
            lk.lock();
        }
        if (--active_ == 0) done_.notify_all();
    }
}

void HostPool::run(int tasks, const std::function<void(int)>& f) {
    std::unique_lock<std::mutex> lk(m_);
    job_ = &f;
    tasks_ = tasks;
    next_ = 0;
    ++gen_;
    cv_.notify_all();
    ++active_;
    while (next_ < tasks_) {
        const int i = next_++;
        lk.unlock();
        f(i);
        lk.lock();
    }
    --active_;
    done_.wait(lk, [&] { return active_ == 0; });
    job_ = nullptr;
    tasks_ = 0;
}

int match_host(bicos_engine* e, const void* const* p0, const size_t* steps0,
               const void* const* p1, const size_t* steps1, int n, int rows, int cols,
               int depth, const BicosConfig& cfg, bool has_nxcorr, float threshold, void* disp,
               void* corr) {
    if (!e) return fail(BICOS_E_ARG, "null engine");
    if (n < 2) return fail(BICOS_E_ARG, "need at least two images");
    if (depth != 1 && depth != 2)
        return fail(BICOS_E_ARG, "bad input depths, only CV_8UC1 and CV_16UC1 are supported");
    if (rows < 0 || cols < 0) return fail(BICOS_E_ARG, "negative image size");
    hipStream_t cs = e->own_stream, ks = e->copy_stream;
    if (rows == 0 || cols == 0)  // validates the configuration, no work
        return match_device(e, nullptr, nullptr, n, rows, cols, (size_t)cols,
                            (size_t)rows * cols, depth, cfg, has_nxcorr, threshold, disp, corr,
                            cs);
    if (!p0 || !p1 || !disp) return fail(BICOS_E_ARG, "null buffer");
    const size_t row_bytes = (size_t)cols * depth;
    for (int t = 0; t < n; ++t) {
        if (!p0[t] || !p1[t]) return fail(BICOS_E_ARG, "null image");
        if ((steps0 && steps0[t] < row_bytes) || (steps1 && steps1[t] < row_bytes))
            return fail(BICOS_E_ARG, "image step smaller than a row");
    }

    // Transfers (measured, tools/host_bench.py): a thread pool gathers each band of the
    // caller's images into a pinned slot and one DMA per band uploads it (5-7 ms per cfg2
    // match, PCIe-bound: 207 MB at 35-42 GB/s while the gathers run; pageable
    // hipMemcpy2DAsync per band and plane: ~11 ms). The maps come down in one copy at the
    // end (band-wise pinned downloads measured no faster).
    // Row bands (every stage is row-local): upload of band b+1 overlaps the
    // match of band b; ~8 bands keep the pipeline tail short without starving the search.
    const int want = rows >= 1024 ? 8 : rows >= 256 ? 4 : rows >= 64 ? 2 : 1;
    const int band_rows = (rows + want - 1) / want;
    const int B = (rows + band_rows - 1) / band_rows;
    const int K = B > 1 ? 3 : 1;  // pinned slots in flight
    const size_t band_bytes = 2 * (size_t)n * band_rows * row_bytes;
    const size_t dsz = has_nxcorr ? 4 : 2, csz = cfg.precision ? 8 : 4;
    const size_t out_off = align_up((size_t)B * band_bytes);
    const size_t corr_off = out_off + align_up((size_t)rows * cols * dsz);
    const size_t total = corr_off + (corr ? (size_t)rows * cols * csz : 0);
    int rc = reserve(e->stage, e->stage_bytes, total, e->device, ks, e->ws_ready);
    if (rc) return rc;
    if (e->pinned_bytes < (size_t)K * band_bytes) {
        if (e->pinned) (void)hipHostFree(e->pinned);
        e->pinned = nullptr;
        e->pinned_bytes = 0;
        rc = check_hip(hipHostMalloc(&e->pinned, (size_t)K * band_bytes, hipHostMallocDefault),
                       "hipHostMalloc(staging)");
        if (rc) return rc;
        e->pinned_bytes = (size_t)K * band_bytes;
    }
    const size_t disp_bytes = (size_t)rows * cols * dsz;
    while ((int)e->events.size() < B) {
        hipEvent_t ev;
        rc = check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
        if (rc) return rc;
        e->events.push_back(ev);
    }
    if (!e->pool) {
        // gather threads (BICOS_HOST_THREADS, default 8): the gathers compete with the DMA
        // for host memory bandwidth; 16 threads measured slower than 3-8 (tools/host_bench.py)
        const unsigned hw = std::thread::hardware_concurrency();
        const char* th = std::getenv("BICOS_HOST_THREADS");
        const unsigned cap = th ? (unsigned)std::max(1, std::atoi(th)) : 8u;
        e->pool.reset(new HostPool((int)std::max(1u, std::min(cap, hw ? hw : 1u))));
    }

    // Round 6 (profiles/host_path_r06.jsonl, host_trace_r06*.txt): each band's
    // upload is split over two copy streams, and the maps come down band by band on a third
    // stream into pinned memory as each band's match ends, then into the caller's buffers by
    // the pool -- 4.40-4.52 ms per cfg2 match against 5.45-5.79 with one upload stream and one
    // download at the end (two rounds interleaved on one box; either change alone was not
    // consistent: 4.86-7.29 / 4.98-5.41 ms). BICOS_HOST_UPLOAD_STREAMS=1 / BICOS_HOST_DL=once:
    // the round-5 pipeline.
    static const bool dl_bands = [] {
        const char* v = std::getenv("BICOS_HOST_DL");
        return !(v && !std::strcmp(v, "once"));
    }();
    static const int up_streams = [] {
        const char* v = std::getenv("BICOS_HOST_UPLOAD_STREAMS");
        return v && std::atoi(v) == 1 ? 1 : 2;
    }();
    if (up_streams == 2) {
        if (!e->copy_stream2) {
            rc = check_hip(hipStreamCreateWithFlags(&e->copy_stream2, hipStreamNonBlocking),
                           "hipStreamCreate");
            if (rc) return rc;
        }
        while ((int)e->events2.size() < B) {
            hipEvent_t ev;
            rc = check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
            if (rc) return rc;
            e->events2.push_back(ev);
        }
        rc = check_hip(hipStreamWaitEvent(e->copy_stream2, e->ws_ready, 0), "hipStreamWaitEvent");
        if (rc) return rc;
    }
    const size_t corr_bytes = corr ? (size_t)rows * cols * csz : 0;
    if (dl_bands) {
        if (!e->dl_stream) {
            rc = check_hip(hipStreamCreateWithFlags(&e->dl_stream, hipStreamNonBlocking),
                           "hipStreamCreate");
            if (rc) return rc;
        }
        const size_t need_out = align_up(disp_bytes) + corr_bytes;
        if (e->pinned_out_bytes < need_out) {
            if (e->pinned_out) (void)hipHostFree(e->pinned_out);
            e->pinned_out = nullptr;
            e->pinned_out_bytes = 0;
            rc = check_hip(hipHostMalloc(&e->pinned_out, need_out, hipHostMallocDefault),
                           "hipHostMalloc(map staging)");
            if (rc) return rc;
            e->pinned_out_bytes = need_out;
        }
        while ((int)e->dl_events.size() < 2 * B) {
            hipEvent_t ev;
            rc = check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
            if (rc) return rc;
            e->dl_events.push_back(ev);
        }
    }
    char* hout_d = dl_bands ? (char*)e->pinned_out : nullptr;
    char* hout_c = dl_bands && corr ? (char*)e->pinned_out + align_up(disp_bytes) : nullptr;

    // BICOS_HOST_TRACE=1: per-phase host timestamps on stderr (tools/host_bench.py)
    static const bool trace = std::getenv("BICOS_HOST_TRACE") != nullptr;
    const auto t_start = std::chrono::steady_clock::now();
    auto stamp = [&](const char* what, int b) {
        if (!trace) return;
        const double us = std::chrono::duration<double, std::micro>(
                              std::chrono::steady_clock::now() - t_start).count();
        std::fprintf(stderr, "[bicos host] %8.1f us  %s %d\n", us, what, b);
    };
    std::vector<std::pair<hipEvent_t, hipEvent_t>> dma_ev;
    // earlier calls (possibly on other streams) may still read the stage / workspace
    rc = check_hip(hipStreamWaitEvent(ks, e->ws_ready, 0), "hipStreamWaitEvent");
    if (rc) return rc;
    char* dev = (char*)e->stage;
    char* dev_disp = dev + out_off;
    char* dev_corr = corr ? dev + corr_off : nullptr;
    for (int b = 0; b < B && rc == BICOS_OK; ++b) {
        const int r0 = b * band_rows;
        const int br = std::min(band_rows, rows - r0);
        const size_t plane = (size_t)br * row_bytes;
        char* slot = (char*)e->pinned + (size_t)(b % K) * band_bytes;
        if (b >= K) {
            rc = check_hip(hipEventSynchronize(e->events[b - K]), "hipEventSynchronize");
            if (!rc && up_streams == 2)
                rc = check_hip(hipEventSynchronize(e->events2[b - K]), "hipEventSynchronize");
            if (rc) break;
        }
        char* band = dev + (size_t)b * band_bytes;
        // 2n planes -> slot [2n][br][cols], dense
        const std::function<void(int)> copy = [&](int i) {
            const bool right = i >= n;
            const int t = right ? i - n : i;
            const size_t step = right ? (steps1 ? steps1[t] : row_bytes)
                                      : (steps0 ? steps0[t] : row_bytes);
            const char* src = (const char*)(right ? p1[t] : p0[t]) + (size_t)r0 * step;
            char* dst = slot + (size_t)i * plane;
            if (step == row_bytes) {
                std::memcpy(dst, src, plane);
            } else {
                for (int r = 0; r < br; ++r)
                    std::memcpy(dst + (size_t)r * row_bytes, src + (size_t)r * step, row_bytes);
            }
        };
        stamp("slot free", b);
        e->pool->run(2 * n, copy);
        stamp("gathered", b);
        hipEvent_t t0 = nullptr, t1 = nullptr;
        if (trace) {
            (void)hipEventCreate(&t0);
            (void)hipEventCreate(&t1);
            (void)hipEventRecord(t0, ks);
        }
        const size_t up = 2 * (size_t)n * plane;
        const size_t first = up_streams == 2 ? (up / 2 + 4095) / 4096 * 4096 : up;
        rc = check_hip(hipMemcpyAsync(band, slot, first, hipMemcpyHostToDevice, ks), "stack upload");
        if (!rc && first < up) {
            rc = check_hip(hipMemcpyAsync(band + first, slot + first, up - first,
                                          hipMemcpyHostToDevice, e->copy_stream2), "stack upload");
            if (!rc) rc = check_hip(hipEventRecord(e->events2[b], e->copy_stream2), "hipEventRecord");
            if (!rc) rc = check_hip(hipStreamWaitEvent(cs, e->events2[b], 0), "hipStreamWaitEvent");
        }
        if (trace) {
            (void)hipEventRecord(t1, ks);
            dma_ev.push_back({t0, t1});
        }
        if (!rc) rc = check_hip(hipEventRecord(e->events[b], ks), "hipEventRecord");
        if (!rc) rc = check_hip(hipStreamWaitEvent(cs, e->events[b], 0), "hipStreamWaitEvent");
        if (!rc)
            rc = match_device(e, band, band + (size_t)n * plane, n, br, cols, (size_t)cols,
                              (size_t)br * cols, depth, cfg, has_nxcorr, threshold,
                              dev_disp + (size_t)r0 * cols * dsz,
                              dev_corr ? dev_corr + (size_t)r0 * cols * csz : nullptr, cs);
        if (!rc && dl_bands) {  // this band's rows of the maps, as soon as they are matched
            hipStream_t ds = e->dl_stream;
            const size_t od = (size_t)r0 * cols * dsz, oc = (size_t)r0 * cols * csz;
            rc = check_hip(hipEventRecord(e->dl_events[2 * b], cs), "hipEventRecord");
            if (!rc) rc = check_hip(hipStreamWaitEvent(ds, e->dl_events[2 * b], 0), "hipStreamWaitEvent");
            if (!rc)
                rc = check_hip(hipMemcpyAsync(hout_d + od, dev_disp + od, (size_t)br * cols * dsz,
                                              hipMemcpyDeviceToHost, ds), "download");
            if (!rc && corr)
                rc = check_hip(hipMemcpyAsync(hout_c + oc, dev_corr + oc, (size_t)br * cols * csz,
                                              hipMemcpyDeviceToHost, ds), "download");
            if (!rc) rc = check_hip(hipEventRecord(e->dl_events[2 * b + 1], ds), "hipEventRecord");
        }
    }
    stamp("bands queued", B);
    if (trace) {
        (void)hipStreamSynchronize(cs);
        stamp("bands matched", B);
    }
    if (!rc && dl_bands) {
        // each band into the caller's buffers as it lands (the pool: row chunks of both maps)
        for (int b = 0; b < B && !rc; ++b) {
            rc = check_hip(hipEventSynchronize(e->dl_events[2 * b + 1]), "hipEventSynchronize");
            if (rc) break;
            const int r0 = b * band_rows;
            const int br = std::min(band_rows, rows - r0);
            const int parts = 8;
            const std::function<void(int)> out = [&](int i) {
                const bool c = i >= parts;
                if (c && !corr) return;
                const size_t esz = c ? csz : dsz;
                const size_t bytes = (size_t)br * cols * esz;
                const size_t chunk = (bytes / parts + 63) / 64 * 64;
                const size_t o = (size_t)(i % parts) * chunk;
                if (o >= bytes) return;
                const size_t base = (size_t)r0 * cols * esz + o;
                std::memcpy((char*)(c ? corr : disp) + base, (c ? hout_c : hout_d) + base,
                            std::min(chunk, bytes - o));
            };
            e->pool->run(2 * parts, out);
        }
    } else if (!rc) {
        rc = check_hip(hipMemcpyAsync(disp, dev_disp, disp_bytes, hipMemcpyDeviceToHost, cs),
                       "download");
        if (!rc && corr)
            rc = check_hip(hipMemcpyAsync(corr, dev_corr, corr_bytes, hipMemcpyDeviceToHost, cs),
                           "download");
    }
    // drain every stream whatever happened: the slots and the stage are reused next call
    const int r1 = check_hip(hipStreamSynchronize(ks), "hipStreamSynchronize");
    if (up_streams == 2) (void)hipStreamSynchronize(e->copy_stream2);
    const int r2 = check_hip(hipStreamSynchronize(cs), "hipStreamSynchronize");
    const int r3 = dl_bands ? check_hip(hipStreamSynchronize(e->dl_stream), "hipStreamSynchronize")
                            : BICOS_OK;
    stamp("downloaded", B);
    for (size_t i = 0; i < dma_ev.size(); ++i) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, dma_ev[i].first, dma_ev[i].second);
        std::fprintf(stderr, "[bicos host] dma %zu: %.3f ms = %.1f GB/s\n", i, ms,
                     band_bytes / (ms * 1e6));
        (void)hipEventDestroy(dma_ev[i].first);
        (void)hipEventDestroy(dma_ev[i].second);
    }
    return rc ? rc : (r1 ? r1 : (r2 ? r2 : r3));
}

namespace {
std::mutex g_engines_lock;
std::map<int, bicos_engine*> g_engines;
}  // namespace

bicos_engine* default_engine(int device) {
    std::lock_guard<std::mutex> g(g_engines_lock);
    auto it = g_engines.find(device);
    if (it != g_engines.end()) return it->second;
    bicos_engine* e = nullptr;
    if (bicos_engine_create(device, &e) != BICOS_OK) return nullptr;
    g_engines[device] = e;
    return e;
}

bool is_default_engine(const bicos_engine* e) {
    std::lock_guard<std::mutex> g(g_engines_lock);
    for (const auto& kv : g_engines)
        if (kv.second == e) return true;
    return false;
}

}  // namespace bicos_impl

// ------------------------------------------------------------- C-ABI: engine

using namespace bicos_impl;

extern "C" {

const char* bicos_last_error(void) { return bicos_impl::last_error(); }

int bicos_engine_create(int device, bicos_engine** out) {
    if (!out) return fail(BICOS_E_ARG, "null out");
    *out = nullptr;
    int count = 0;
    int rc = check_hip(hipGetDeviceCount(&count), "hipGetDeviceCount");
    if (rc) return rc;
    if (device < 0 || device >= count) return fail(BICOS_E_ARG, "no such HIP device");
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    auto* e = new bicos_engine();
    e->device = device;
    int lds = 0;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) ==
            hipSuccess &&
        lds > 0) {
        // keep the per-workgroup right-row stage <= 64 KiB so >= 2 workgroups fit per CU
        e->max_lds = lds < 64 * 1024 ? lds : 64 * 1024;
        e->lds_limit = lds;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cus > 0)
        e->cus = cus;
    rc = check_hip(hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking), "hipStreamCreate");
    if (!rc)
        rc = check_hip(hipStreamCreateWithFlags(&e->copy_stream, hipStreamNonBlocking),
                       "hipStreamCreate");
    if (!rc)
        rc = check_hip(hipEventCreateWithFlags(&e->ws_ready, hipEventDisableTiming),
                       "hipEventCreate");
    (void)hipSetDevice(cur);
    if (rc) {
        if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
        if (e->copy_stream) (void)hipStreamDestroy(e->copy_stream);
    if (e->ws_ready) (void)hipEventDestroy(e->ws_ready);
        delete e;
        return rc;
    }
    *out = e;
    return BICOS_OK;
}

bicos_engine* bicos_engine_default(int device) { return default_engine(device); }

void bicos_engine_destroy(bicos_engine* e) {
    if (!e) return;
    if (is_default_engine(e)) return;  // the process-wide engines live until exit
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(e->device);
    (void)hipDeviceSynchronize();
    // workspaces come from the stream-ordered allocator (reserve)
    if (e->ws) (void)hipFreeAsync(e->ws, e->own_stream);
    if (e->stage) (void)hipFreeAsync(e->stage, e->own_stream);
    (void)hipStreamSynchronize(e->own_stream);
    if (e->pinned) (void)hipHostFree(e->pinned);
    for (hipEvent_t ev : e->events) (void)hipEventDestroy(ev);
    if (e->gather_pinned) (void)hipHostFree(e->gather_pinned);
    for (hipEvent_t ev : e->gather_events) (void)hipEventDestroy(ev);
    if (e->pinned_out) (void)hipHostFree(e->pinned_out);
    for (hipEvent_t ev : e->dl_events) (void)hipEventDestroy(ev);
    if (e->dl_stream) (void)hipStreamDestroy(e->dl_stream);
    if (e->copy_stream2) (void)hipStreamDestroy(e->copy_stream2);
    for (hipEvent_t ev : e->events2) (void)hipEventDestroy(ev);
    e->pool.reset();
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    if (e->copy_stream) (void)hipStreamDestroy(e->copy_stream);
    (void)hipSetDevice(cur);
    delete e;
}

int bicos_engine_tune(bicos_engine* e, int variant, int col0_per_lane, int waves, int split) {
    if (!e) return fail(BICOS_E_ARG, "null engine");
    if (variant >= 64 && variant <= 68) {
        // matrix-core search (64 auto keys, 65 one product + xor keys, 66 two products, 67
        // xor keys for first-minimum searches too, no FK keys, 68 packed keys where they
        // apply -- the automatic choice);
        // col0_per_lane = 32-column tiles per wave
        if (col0_per_lane != 0 && col0_per_lane != 2 && col0_per_lane != 4 && col0_per_lane != 8)
            return fail(BICOS_E_ARG, "variant 64-68: tiles per wave 2|4|8");
        if (waves < 0 || waves > 8) return fail(BICOS_E_ARG, "waves 1..8");
        if (split < 0 || split > 160) return fail(BICOS_E_ARG, "variant 64-68: split = LDS KiB 0..160");
        e->tune_variant = variant;
        e->tune_R = col0_per_lane;
        e->tune_waves = waves;
        e->tune_split = split;
        return BICOS_OK;
    }
    if (variant != 0 && variant != 16) return fail(BICOS_E_ARG, "variant 0|16|64..68");
    if (col0_per_lane != 0 && col0_per_lane != 2 && col0_per_lane != 4)
        return fail(BICOS_E_ARG, "col0_per_lane: 2|4 (variant 16)");
    if (waves < 0 || waves > 8) return fail(BICOS_E_ARG, "waves 1..8");
    if (split != 0 && split != 1 && split != 2 && split != 4 && split != 8)
        return fail(BICOS_E_ARG, "split 1|2|4|8");
    if (split > 1 && (waves ? waves : 8) % split)
        return fail(BICOS_E_ARG, "split needs waves divisible by split");
    e->tune_variant = variant;
    e->tune_R = col0_per_lane;
    e->tune_waves = waves;
    e->tune_split = split;
    return BICOS_OK;
}

int bicos_descriptor_words(int n, int mode) {
    if (n < 2) return fail(BICOS_E_ARG, "need at least two images");
    const int w = descriptor_words(n, mode ? 1 : 0);
    if (w < 0) return fail(BICOS_E_BITS, "input stacks too large");
    return w;
}

int bicos_output_type(const BicosConfig* cfg, int has_nxcorr) {
    (void)cfg;
    return has_nxcorr ? BICOS_CV_32F : BICOS_CV_16S;
}

size_t bicos_desc_pitch(int cols, int words) {
    return ((size_t)cols * words + 3) / 4 * 4;
}

namespace {
int match_device_entry(bicos_engine* e, const void* stack0, const void* stack1, int n, int rows,
                       int cols, size_t row_pitch, size_t plane_pitch, int depth,
                       const BicosConfig* cfg, int has_nxcorr, void* disparity, void* corrmap,
                       void* stream, bool disp_i16) {
    if (!cfg) return fail(BICOS_E_ARG, "null config");
    if (!e) return fail(BICOS_E_ARG, "null engine");
    try {
        // the engine's workspace may be shared with other threads (the default engine is):
        // enqueueing is serialised per engine, the GPU work is ordered through ws_ready
        std::lock_guard<std::mutex> g(e->lock);
        // reference src/pybicos_c.cpp:59-61: a negative threshold keeps the default 0.5
        const float thr = cfg->nxcorr_threshold >= 0 ? cfg->nxcorr_threshold : 0.5f;
        return match_device(e, stack0, stack1, n, rows, cols, row_pitch, plane_pitch, depth, *cfg,
                            has_nxcorr != 0, thr, disparity, corrmap, (hipStream_t)stream, disp_i16);
    } catch (const std::exception& ex) {
        return fail(BICOS_E_INTERNAL, ex.what());
    } catch (...) {
        return fail(BICOS_E_INTERNAL, "unknown exception");
    }
}
}  // namespace

int bicos_match_device(bicos_engine* e, const void* stack0, const void* stack1, int n, int rows,
                       int cols, size_t row_pitch, size_t plane_pitch, int depth,
                       const BicosConfig* cfg, int has_nxcorr, void* disparity, void* corrmap,
                       void* stream) {
    return match_device_entry(e, stack0, stack1, n, rows, cols, row_pitch, plane_pitch, depth, cfg,
                              has_nxcorr, disparity, corrmap, stream, false);
}

int bicos_match_device_i16(bicos_engine* e, const void* stack0, const void* stack1, int n, int rows,
                           int cols, size_t row_pitch, size_t plane_pitch, int depth,
                           const BicosConfig* cfg, int has_nxcorr, void* disparity, void* corrmap,
                           void* stream) {
    return match_device_entry(e, stack0, stack1, n, rows, cols, row_pitch, plane_pitch, depth, cfg,
                              has_nxcorr, disparity, corrmap, stream, true);
}

int bicos_match_plan(bicos_engine* e, const void* stack0, const void* stack1, int n, int rows,
                     int cols, size_t row_pitch, size_t plane_pitch, int depth,
                     const BicosConfig* cfg, int has_nxcorr) {
    if (!cfg) return fail(BICOS_E_ARG, "null config");
    if (n < 2) return fail(BICOS_E_ARG, "need at least two images");
    if (depth != 1 && depth != 2) return fail(BICOS_E_ARG, "bad input depth");
    if (descriptor_words(n, cfg->mode ? 1 : 0) < 0) return fail(BICOS_E_BITS, "input stacks too large");
    return match_plan(e, n, rows, cols, row_pitch, plane_pitch, depth, *cfg, has_nxcorr != 0,
                      stack0, stack1);
}

int bicos_search_agree_device(bicos_engine* e, const uint32_t* desc0, const uint32_t* desc1,
                              const void* stack0, const void* stack1, int n, int rows, int cols,
                              size_t row_pitch, size_t plane_pitch, int depth,
                              const BicosConfig* cfg, int has_nxcorr, void* disparity,
                              void* corrmap, void* stream) {
    if (!cfg) return fail(BICOS_E_ARG, "null config");
    if (!e) return fail(BICOS_E_ARG, "null engine");
    if (rows > 0 && cols > 0 && (!desc0 || !desc1)) return fail(BICOS_E_ARG, "null descriptors");
    try {
        std::lock_guard<std::mutex> g(e->lock);
        const float thr = cfg->nxcorr_threshold >= 0 ? cfg->nxcorr_threshold : 0.5f;
        return match_device(e, stack0, stack1, n, rows, cols, row_pitch, plane_pitch, depth, *cfg,
                            has_nxcorr != 0, thr, disparity, corrmap, (hipStream_t)stream, false,
                            desc0, desc1);
    } catch (const std::exception& ex) {
        return fail(BICOS_E_INTERNAL, ex.what());
    } catch (...) {
        return fail(BICOS_E_INTERNAL, "unknown exception");
    }
}

int bicos_match_host(bicos_engine* e, const void* const* stack0, const void* const* stack1, int n,
                     int rows, int cols, size_t step, int depth, const BicosConfig* cfg,
                     int has_nxcorr, void* disparity, void* corrmap) {
    if (!cfg) return fail(BICOS_E_ARG, "null config");
    if (n < 0) return fail(BICOS_E_ARG, "negative stack size");
    try {
        if (!e) {
            int dev = 0;
            int rc = check_hip(hipGetDevice(&dev), "hipGetDevice");
            if (rc) return rc;
            e = default_engine(dev);
            if (!e) return BICOS_E_HIP;  // bicos_last_error says why
        }
        std::lock_guard<std::mutex> g(e->lock);
        // reference src/pybicos_c.cpp:59-61: a negative threshold keeps the default 0.5
        const float thr = cfg->nxcorr_threshold >= 0 ? cfg->nxcorr_threshold : 0.5f;
        const std::vector<size_t> steps((size_t)n, step ? step : (size_t)(cols > 0 ? cols : 0) * depth);
        return match_host(e, stack0, steps.data(), stack1, steps.data(), n, rows, cols, depth, *cfg,
                          has_nxcorr != 0, thr, disparity, corrmap);
    } catch (const std::exception& ex) {
        return fail(BICOS_E_INTERNAL, ex.what());
    } catch (...) {
        return fail(BICOS_E_INTERNAL, "unknown exception");
    }
}

int bicos_transform_device(const void* stack, int n, int rows, int cols, size_t row_pitch,
                           size_t plane_pitch, int depth, int mode, int words, uint32_t* desc,
                           void* stream) {
    if (n < 2) return fail(BICOS_E_ARG, "need at least two images");
    if (depth != 1 && depth != 2) return fail(BICOS_E_ARG, "bad input depth");
    if (words != 1 && words != 2 && words != 4 && words != 8)
        return fail(BICOS_E_ARG, "words must be 1, 2, 4 or 8");
    const int need = descriptor_words(n, mode ? 1 : 0);
    if (need < 0 || need > words) return fail(BICOS_E_BITS, "descriptor too narrow for n");
    uint32_t span = 0;
    if (int rc0 = stack_span(n, rows, cols, row_pitch, plane_pitch, depth, &span)) return rc0;
    bicos_hip::TransformArgs ta{stack, nullptr, desc, nullptr, n, rows, cols,
                                row_pitch, plane_pitch, bicos_desc_pitch(cols, words), 0, span};
    return check_hip(bicos_hip::launch_transform(ta, depth, mode ? 1 : 0, words, (hipStream_t)stream),
                     "transform launch");
}

int bicos_search_device(bicos_engine* e, const uint32_t* desc0, const uint32_t* desc1, int rows,
                        int cols, int words, int flags, int max_lr_diff, int16_t* out,
                        void* stream) {
    if (words != 1 && words != 2 && words != 4 && words != 8)
        return fail(BICOS_E_ARG, "words must be 1, 2, 4 or 8");
    if (cols > 32767) return fail(BICOS_E_ARG, "image width exceeds 32767");
    if (rows <= 0 || cols <= 0) return BICOS_OK;
    hipStream_t st = (hipStream_t)stream;
    const size_t dpitch = bicos_desc_pitch(cols, words);
    const bool nodupes = (flags & 1) != 0;
    const int bits = (flags >> 16) & 0x1FF;  // 0 = all descriptor bits may be set
    const bool mx = use_mx(e);
    const bicos_hip::SearchGeometry g = mx ? bicos_hip::SearchGeometry{} : geometry(e, rows, cols, words);
    if (!(flags & 2)) {
        bicos_hip::SearchArgs sa{desc0, desc1, out, rows, cols, dpitch, (size_t)cols, 0, 0, 0};
        if (mx)
            return check_hip(bicos_hip::launch_search_mx(sa, mx_geometry(e, rows, cols, words, bits),
                                                         words, nodupes, st),
                             "search launch");
        return check_hip(bicos_hip::launch_search(sa, g, words, nodupes, st), "search launch");
    }
    if (mx && !nodupes && lr_one_pass() && bicos_hip::search_lr_eligible(words, bits, cols)) {
        bicos_hip::SearchArgs sa{desc0, desc1, out, rows, cols, dpitch, (size_t)cols, 0, 0, 0};
        return check_hip(bicos_hip::launch_search_lr(sa, words, bits, max_lr_diff, st),
                         "consistency search launch");
    }
    if (!e) return fail(BICOS_E_ARG, "consistency search needs an engine workspace");
    std::lock_guard<std::mutex> lk(e->lock);  // the workspace may be shared (default engine)
    const size_t map16 = align_up((size_t)rows * cols * 2);
    const bool dense = mx && reverse_compacted(true) && dense_rows();
    const size_t vpitch = valid_pitch(cols);
    const size_t vbytes = dense ? align_up((size_t)rows * vpitch) : 0;
    int rc = reserve(e->ws, e->ws_bytes, 2 * map16 + vbytes, e->device, st, e->ws_ready);
    if (rc) return rc;
    rc = check_hip(hipStreamWaitEvent(st, e->ws_ready, 0), "hipStreamWaitEvent");
    if (rc) return rc;
    struct MarkUse {
        hipEvent_t ev;
        hipStream_t st;
        ~MarkUse() { (void)hipEventRecord(ev, st); }
    } mark{e->ws_ready, st};
    int16_t* fwd = (int16_t*)e->ws;
    int16_t* rev = (int16_t*)((char*)e->ws + map16);
    uint8_t* valid = dense ? (uint8_t*)e->ws + 2 * map16 : nullptr;
    bicos_hip::SearchArgs fa{desc0, desc1, fwd, rows, cols, dpitch, (size_t)cols, 1, 0, 0};
    bicos_hip::SearchArgs ra{desc1, desc0, rev, rows, cols, dpitch, (size_t)cols, 1, 0, 0};
    if (mx) {
        const bicos_hip::MxGeometry gm = mx_geometry(e, rows, cols, words, bits);
        fa.row_valid = ra.row_valid = valid;
        fa.valid_pitch = ra.valid_pitch = vpitch;
        rc = check_hip(bicos_hip::launch_search_mx(fa, gm, words, nodupes, st), "search launch");
        if (rc) return rc;
        if (reverse_compacted(true)) {
            ra.keep = fwd;
            ra.keep_pitch = (size_t)cols;
        }
        rc = check_hip(bicos_hip::launch_search_mx(ra, gm, words, nodupes, st),
                       "reverse search launch");
    } else {
        rc = check_hip(bicos_hip::launch_search(fa, g, words, nodupes, st), "search launch");
        if (rc) return rc;
        rc = check_hip(bicos_hip::launch_search(ra, g, words, nodupes, st), "reverse search launch");
    }
    if (rc) return rc;
    bicos_hip::ConsistencyArgs ca{fwd, rev, out, rows, cols, (size_t)cols, max_lr_diff};
    return check_hip(bicos_hip::launch_consistency(ca, st), "consistency launch");
}

static int agree_common(bool sub, const int16_t* raw, const void* stack0, const void* stack1,
                        int n, int rows, int cols, size_t row_pitch, size_t plane_pitch, int depth,
                        float threshold, float step, int has_minvar, float minvar_scaled,
                        float* out, void* corrmap, void* stream, bool dbl = false) {
    if (n < 2) return fail(BICOS_E_ARG, "need at least two images");
    if (n > 65 && sub) return fail(BICOS_E_ARG, "subpixel supports n <= 65");
    if (depth != 1 && depth != 2) return fail(BICOS_E_ARG, "bad input depth");
    if (sub && !(step > 0 && std::isfinite(step)))
        return fail(BICOS_E_ARG, "subpixel_step must be a positive finite number");
    const int nsteps = sub ? subpixel_steps(step) : 0;
    if (sub && !nsteps)
        return fail(BICOS_E_ARG, "subpixel_step too small (more than 65536 interpolation steps)");
    bicos_hip::AgreeArgs aa{};
    aa.raw = raw;
    aa.raw_pitch = (size_t)cols;
    aa.stack0 = stack0;
    aa.stack1 = stack1;
    aa.n = n;
    aa.rows = rows;
    aa.cols = cols;
    aa.row_pitch = row_pitch;
    aa.plane_pitch = plane_pitch;
    aa.threshold = threshold;
    aa.step = step;
    aa.nsteps = nsteps;
    aa.has_minvar = has_minvar;
    aa.minvar = minvar_scaled;
    aa.out = out;
    aa.out_f32 = 1;
    aa.corrmap = corrmap;
    if (int rc0 = stack_span(n, rows, cols, row_pitch, plane_pitch, depth, &aa.stack_bytes)) return rc0;
    hipStream_t st = (hipStream_t)stream;
    return sub ? check_hip(bicos_hip::launch_subpixel(aa, depth, dbl, st), "subpixel launch")
               : check_hip(bicos_hip::launch_agree(aa, depth, dbl, st), "agree launch");
}

int bicos_agree_stage_device(const int16_t* raw, const void* stack0, const void* stack1, int n,
                             int rows, int cols, size_t row_pitch, size_t plane_pitch, int depth,
                             float threshold, float step, int has_minvar, float minvar_scaled,
                             int precision, float* out, void* corrmap, void* stream) {
    return agree_common(step > 0, raw, stack0, stack1, n, rows, cols, row_pitch, plane_pitch,
                        depth, threshold, step, has_minvar, minvar_scaled, out, corrmap, stream,
                        precision != 0);
}

int bicos_agree_device(const int16_t* raw, const void* stack0, const void* stack1, int n, int rows,
                       int cols, size_t row_pitch, size_t plane_pitch, int depth, float threshold,
                       int has_minvar, float minvar_scaled, float* out, float* corrmap,
                       void* stream) {
    return agree_common(false, raw, stack0, stack1, n, rows, cols, row_pitch, plane_pitch, depth,
                        threshold, 0.f, has_minvar, minvar_scaled, out, corrmap, stream);
}

int bicos_subpixel_device(const int16_t* raw, const void* stack0, const void* stack1, int n,
                          int rows, int cols, size_t row_pitch, size_t plane_pitch, int depth,
                          float threshold, float step, int has_minvar, float minvar_scaled,
                          float* out, float* corrmap, void* stream) {
    return agree_common(true, raw, stack0, stack1, n, rows, cols, row_pitch, plane_pitch, depth,
                        threshold, step, has_minvar, minvar_scaled, out, corrmap, stream);
}

const char* bicos_build_info(void) {
    return "libbicos_amd: gfx950 HIP kernels (transform, mx search: FP4 MFMA Hamming products "
           "with argmin keys in the accumulator [default], LDS-broadcast popcount/argmin VALU "
           "search, NXC agree/subpixel), -O3 -ffp-contract=off";
}

}  // extern "C"

// --------------------------------------------------------------- C++ API

namespace BICOS {

size_t HipImage::elem_size(int type) {
    switch (type) {
        case U8: return 1;
        case U16:
        case S16: return 2;
        case F32: return 4;
        case F64: return 8;
    }
    throw Exception("unsupported image type " + std::to_string(type));
}

HipImage::HipImage(int rows, int cols, int type, void* data, size_t step, Memory mem)
    : _data(data), _rows(rows), _cols(cols), _type(type), _mem(mem) {
    _step = step ? step : (size_t)cols * elem_size(type);
}

void HipImage::create(int rows, int cols, int type, Memory mem) {
    // like cv::Mat::create: a no-op when the header already describes a dense buffer of this
    // size and type (owned or a view of the caller's memory), so results can be written
    // straight into caller-provided buffers
    if (_data && _rows == rows && _cols == cols && _type == type && _mem == mem &&
        _step == (size_t)cols * elem_size(type))
        return;
    const size_t step = (size_t)cols * elem_size(type);
    const size_t bytes = step * rows;
    void* p = nullptr;
    if (mem == Memory::Host) {
        p = std::malloc(bytes ? bytes : 1);
        if (!p) throw Exception("out of host memory");
        _owner = std::shared_ptr<void>(p, [](void* q) { std::free(q); });
    } else {
        if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) throw Exception("hipMalloc failed");
        _owner = std::shared_ptr<void>(p, [](void* q) { (void)hipFree(q); });
    }
    _data = p;
    _rows = rows;
    _cols = cols;
    _type = type;
    _step = step;
    _mem = mem;
}

HipImage HipImage::download() const {
    if (_mem == Memory::Host) return *this;
    Image h = allocate(_rows, _cols, _type, Memory::Host);
    if (!empty() &&
        hipMemcpy2D(h._data, h._step, _data, _step, (size_t)_cols * elemSize(), _rows,
                    hipMemcpyDeviceToHost) != hipSuccess)
        throw Exception("download failed");
    return h;
}

static void throw_rc(int rc) {
    if (rc != BICOS_OK) throw Exception(bicos_impl::last_error());
}

// reference src/impl/cpu.cpp:100-159 (validation, dispatch) + src/lib.cpp:31-49
void match(const std::vector<Image>& stack0, const std::vector<Image>& stack1, Image& disparity,
           Config cfg, Image* corrmap, hipStream_t stream) {
    impl::hip::match(stack0, stack1, disparity, cfg, corrmap, stream);
}

// the backend seam (bicos/hip.hpp; reference include/cpu.hpp:27-33, include/cuda.hpp:27-34)
void impl::hip::match(const std::vector<Image>& stack0, const std::vector<Image>& stack1,
                      Image& disparity, Config cfg, Image* corrmap, hipStream_t stream) {
    const size_t n = stack0.size();
    if (n < 2) throw Exception("need at least two images");
    if (stack1.size() != n) throw Exception("stacks differ in length");
    const Image& f = stack0.front();
    if (f.type() != U8 && f.type() != U16)
        throw Exception("bad input depths, only CV_8UC1 and CV_16UC1 are supported");
    const Memory mem = f.memory();
    for (const auto* s : {&stack0, &stack1})
        for (const Image& im : *s)
            if (im.rows() != f.rows() || im.cols() != f.cols() || im.type() != f.type() ||
                im.memory() != mem)
                throw Exception("all images must share size, type and memory");
    const int rows = f.rows(), cols = f.cols();
    const int depth = (int)f.elemSize();

    BicosConfig c{};
    const bool has_nxcorr = cfg.nxcorr_threshold.has_value();
    c.nxcorr_threshold = has_nxcorr ? *cfg.nxcorr_threshold : 0.5f;
    c.subpixel_step = cfg.subpixel_step ? *cfg.subpixel_step : -1.f;
    c.min_variance = cfg.min_variance ? *cfg.min_variance : -1.f;
    c.mode = cfg.mode == TransformMode::FULL ? 1 : 0;
    c.precision = cfg.precision == Precision::DOUBLE ? 1 : 0;
    if (auto* cons = std::get_if<Variant::Consistency>(&cfg.variant)) {
        c.variant_type = 1;
        c.max_lr_diff = cons->max_lr_diff;
        c.no_dupes = cons->no_dupes;
    }
    if (cfg.subpixel_step && !(*cfg.subpixel_step > 0))
        throw Exception("subpixel_step must be a positive finite number");
    if (cfg.min_variance && *cfg.min_variance < 0) c.min_variance = -1.f;

    int dev = 0;
    (void)hipGetDevice(&dev);
    bicos_engine* e = bicos_impl::default_engine(dev);
    if (!e) throw Exception(bicos_impl::last_error());
    std::lock_guard<std::mutex> g(e->lock);
    hipStream_t st = mem == Memory::Host ? e->own_stream : stream;
    const int dtype = has_nxcorr ? F32 : S16;
    const bool dbl = c.precision != 0;
    const bool want_corr = corrmap && has_nxcorr;

    if (mem == Memory::Host) {
        // banded, pipelined upload -> match -> download (bicos_impl::match_host)
        std::vector<const void*> p0(n), p1(n);
        std::vector<size_t> st0(n), st1(n);
        for (size_t t = 0; t < n; ++t) {
            p0[t] = stack0[t].data();
            p1[t] = stack1[t].data();
            st0[t] = stack0[t].step();
            st1[t] = stack1[t].step();
        }
        disparity.create(rows, cols, dtype, Memory::Host);
        if (want_corr) corrmap->create(rows, cols, dbl ? F64 : F32, Memory::Host);
        throw_rc(bicos_impl::match_host(e, p0.data(), st0.data(), p1.data(), st1.data(), (int)n,
                                        rows, cols, depth, c, has_nxcorr, c.nxcorr_threshold,
                                        disparity.data(), want_corr ? corrmap->data() : nullptr));
        return;
    }

    // the planar device stacks the kernels read
    const size_t elem = (size_t)depth;
    const void* s0 = nullptr;
    const void* s1 = nullptr;
    size_t row_pitch = (size_t)cols, plane_pitch = (size_t)rows * cols;
    auto uniform = [&](const std::vector<Image>& s, size_t& rp, size_t& pp) {
        // zero-copy when the images already form one planar buffer with a common pitch
        if (s[0].step() % elem) return false;
        rp = s[0].step() / elem;
        const char* b = (const char*)s[0].data();
        if (n < 2) return false;
        const ptrdiff_t d = (const char*)s[1].data() - b;
        if (d <= 0 || d % (ptrdiff_t)elem) return false;
        for (size_t t = 0; t < n; ++t)
            if (s[t].step() != s[0].step() || (const char*)s[t].data() != b + (ptrdiff_t)t * d)
                return false;
        pp = (size_t)d / elem;
        return pp >= (size_t)rows * rp;
    };
    size_t rp0 = 0, pp0 = 0, rp1 = 0, pp1 = 0;
    // staged rows start 64-byte aligned: no two copies share a dword and the pitches suit
    // the aligned (LDS-staged) agree kernel
    const size_t stage_row = ((size_t)cols * elem + 63) & ~(size_t)63;
    const size_t plane_bytes = (size_t)rows * stage_row;
    if (uniform(stack0, rp0, pp0) && uniform(stack1, rp1, pp1) && rp0 == rp1 && pp0 == pp1) {
        s0 = stack0[0].data();
        s1 = stack1[0].data();
        row_pitch = rp0;
        plane_pitch = pp0;
    } else if (rows > 0 && cols > 0) {
        throw_rc(reserve(e->stage, e->stage_bytes, 2 * n * plane_bytes, e->device, st, e->ws_ready));
        throw_rc(check_hip(hipStreamWaitEvent(st, e->ws_ready, 0), "hipStreamWaitEvent"));
        char* dst = (char*)e->stage;
        const hipMemcpyKind kind = hipMemcpyDeviceToDevice;
        for (size_t t = 0; t < n; ++t) {
            throw_rc(check_hip(hipMemcpy2DAsync(dst + t * plane_bytes, stage_row,
                                                stack0[t].data(), stack0[t].step(), cols * elem,
                                                rows, kind, st),
                               "stack upload"));
            throw_rc(check_hip(hipMemcpy2DAsync(dst + (n + t) * plane_bytes, stage_row,
                                                stack1[t].data(), stack1[t].step(), cols * elem,
                                                rows, kind, st),
                               "stack upload"));
        }
        s0 = dst;
        s1 = dst + n * plane_bytes;
        row_pitch = stage_row / elem;
        plane_pitch = plane_bytes / elem;
    }

    disparity.create(rows, cols, dtype, Memory::Device);
    if (want_corr) corrmap->create(rows, cols, dbl ? F64 : F32, Memory::Device);
    throw_rc(bicos_impl::match_device(e, s0, s1, (int)n, rows, cols, row_pitch, plane_pitch, depth,
                                      c, has_nxcorr, c.nxcorr_threshold, disparity.data(),
                                      want_corr ? corrmap->data() : nullptr, st));
}

}  // namespace BICOS
