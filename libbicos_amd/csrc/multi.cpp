// multi.cpp -- single-process multi-GPU match of one frame.
//
// The reference has no multi-GPU path; this is the in-process form of the row-band split
// that bench.py / distributed.py run with one process per GPU. Every stage of the match is
// row-local (transform: one pixel's own samples; search: one row; agree / subpixel: one
// row of both stacks), so a frame splits into contiguous row bands with no halo and the
// band maps, put back in row order, are byte-identical to the whole-frame maps.
//
//   bicos_match_host_multi    host frame in, host maps out: one host thread per band, each
//                             driving the banded host pipeline (match_host) of its GPU over
//                             that GPU's own PCIe link; the maps land in the caller's
//                             buffers at the band's row offset. No device-to-device traffic.
//   bicos_match_bands_device  bands already resident on their GPUs: each GPU matches its
//                             band, the maps are gathered to devices[0] with peer copies
//                             over xGMI (one copy per band and map, on the band's stream).
//                             In one process a gather IS a set of peer DMAs; RCCL would
//                             issue the same copies behind a communicator (its ncclGather
//                             is what the one-process-per-GPU bench uses).
#include "engine.hpp"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace bicos_impl {
namespace {

// rows [begin, end) of band b of `bands` (sizes differ by <= 1 row; the first rows % bands
// bands get the extra row -- distributed.band_rows)
void band_range(int rows, int bands, int b, int& begin, int& end) {
    const int base = rows / bands, extra = rows % bands;
    begin = b * base + std::min(b, extra);
    end = begin + base + (b < extra ? 1 : 0);
}

int check_devices(const int* devices, int ndev) {
    if (!devices || ndev <= 0) return fail(BICOS_E_ARG, "need at least one device");
    int count = 0;
    int rc = check_hip(hipGetDeviceCount(&count), "hipGetDeviceCount");
    if (rc) return rc;
    for (int b = 0; b < ndev; ++b)
        if (devices[b] < 0 || devices[b] >= count)
            return fail(BICOS_E_ARG, "device index out of range");
    return BICOS_OK;
}

// the first failure of the band workers, message included (bicos_last_error is per thread)
struct FirstError {
    std::mutex m;
    int code = BICOS_OK;
    std::string msg;
    void note(int rc) {
        if (rc == BICOS_OK) return;
        std::lock_guard<std::mutex> g(m);
        if (code == BICOS_OK) {
            code = rc;
            msg = last_error();
        }
    }
    int raise() { return code == BICOS_OK ? BICOS_OK : fail(code, msg); }
};

// Stage slots of one band's maps, appended at `off` (which advances past them): the
// disparity map, then (csz != 0) the corrmap, each 256-byte aligned with 256 bytes of slack.
// The reservation and the enqueue loop of bicos_match_bands_device both walk the bands with
// this one function, so the bytes reserved always cover the offsets written.
void band_stage_offsets(size_t& off, int rows, int cols, size_t dsz, size_t csz, size_t* od,
                        size_t* oc) {
    auto slot = [&](size_t bytes) {
        const size_t at = off;
        off = (off + bytes + 256 + 255) / 256 * 256;
        return at;
    };
    *od = slot((size_t)rows * cols * dsz);
    *oc = csz ? slot((size_t)rows * cols * csz) : 0;
}

// Let `peer` read and write memory of `owner`'s default stream-ordered pool (hipMallocAsync,
// which peer access does not cover). No error string: a refusal is not an error of the match.
bool share_pool(int owner, int peer) {
    hipMemPool_t pool = nullptr;
    if (hipDeviceGetDefaultMemPool(&pool, owner) != hipSuccess) return false;
    hipMemAccessDesc d{};
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = peer;
    d.flags = hipMemAccessFlagsProtReadWrite;
    return hipMemPoolSetAccess(pool, &d, 1) == hipSuccess;
}

// Direct xGMI peer DMA from `dev` (the current device) into `root`'s maps, all or nothing
// (ADVICE r04): peer access in both directions AND each device's pool open to the other. A
// partial grant -- peer access on, a pool closed -- would let the copy engine DMA into memory
// it has no mapping for, so then the peer access this call enabled is switched off again and
// the caller copies through pinned host memory instead. Nothing here sets the error string.
bool enable_peer_path(int dev, int root) {
    int fwd = 0, back = 0;
    bool ok = hipDeviceCanAccessPeer(&fwd, dev, root) == hipSuccess && fwd &&
              hipDeviceCanAccessPeer(&back, root, dev) == hipSuccess && back;
    bool enabled_here = false;
    if (ok) {
        const hipError_t pe = hipDeviceEnablePeerAccess(root, 0);
        enabled_here = pe == hipSuccess;
        ok = pe == hipSuccess || pe == hipErrorPeerAccessAlreadyEnabled;
    }
    ok = ok && share_pool(dev, root) && share_pool(root, dev);
    if (!ok && enabled_here) (void)hipDeviceDisablePeerAccess(root);
    (void)hipGetLastError();  // clear a sticky refusal / "already enabled"
    return ok;
}

float nxc_threshold(const BicosConfig& cfg) {
    // reference src/pybicos_c.cpp:59-61: a negative threshold keeps the default 0.5
    return cfg.nxcorr_threshold >= 0 ? cfg.nxcorr_threshold : 0.5f;
}

}  // namespace
}  // namespace bicos_impl

using namespace bicos_impl;

extern "C" int bicos_match_host_multi(const int* devices, int ndev, const void* const* stack0,
                                      const void* const* stack1, int n, int rows, int cols,
                                      size_t step, int depth, const BicosConfig* cfg,
                                      int has_nxcorr, void* disparity, void* corrmap) {
    if (!cfg) return fail(BICOS_E_ARG, "null config");
    if (n < 2) return fail(BICOS_E_ARG, "need at least two images");
    if (depth != 1 && depth != 2)
        return fail(BICOS_E_ARG, "bad input depths, only CV_8UC1 and CV_16UC1 are supported");
    if (rows < 0 || cols < 0) return fail(BICOS_E_ARG, "negative image size");
    try {
        int rc = check_devices(devices, ndev);
        if (rc) return rc;
        const int bands = std::max(1, std::min(ndev, rows));
        const size_t row_bytes = (size_t)cols * depth;
        const size_t pitch = step ? step : row_bytes;
        const size_t dsz = has_nxcorr ? 4 : 2, csz = cfg->precision ? 8 : 4;
        const float thr = nxc_threshold(*cfg);
        FirstError err;
        auto run = [&](int b) {
            try {
                int r0 = 0, r1 = rows;
                if (rows > 0) band_range(rows, bands, b, r0, r1);
                bicos_engine* e = default_engine(devices[b]);
                if (!e) return err.note(BICOS_E_HIP);
                std::vector<const void*> p0((size_t)n), p1((size_t)n);
                for (int t = 0; t < n; ++t) {
                    p0[t] = stack0 && stack0[t] ? (const char*)stack0[t] + (size_t)r0 * pitch : nullptr;
                    p1[t] = stack1 && stack1[t] ? (const char*)stack1[t] + (size_t)r0 * pitch : nullptr;
                }
                const std::vector<size_t> steps((size_t)n, pitch);
                void* d = disparity ? (char*)disparity + (size_t)r0 * cols * dsz : nullptr;
                void* c = corrmap ? (char*)corrmap + (size_t)r0 * cols * csz : nullptr;
                std::lock_guard<std::mutex> g(e->lock);
                int cur = 0;
                (void)hipGetDevice(&cur);
                int r = check_hip(hipSetDevice(devices[b]), "hipSetDevice");
                if (!r)
                    r = match_host(e, p0.data(), steps.data(), p1.data(), steps.data(), n, r1 - r0,
                                   cols, depth, *cfg, has_nxcorr != 0, thr, d, c);
                (void)hipSetDevice(cur);
                err.note(r);
            } catch (const std::exception& ex) {
                err.note(fail(BICOS_E_INTERNAL, ex.what()));
            }
        };
        if (bands == 1) {
            run(0);
        } else {
            std::vector<std::thread> th;
            for (int b = 1; b < bands; ++b) th.emplace_back(run, b);
            run(0);
            for (auto& t : th) t.join();
        }
        return err.raise();
    } catch (const std::exception& ex) {
        return fail(BICOS_E_INTERNAL, ex.what());
    } catch (...) {
        return fail(BICOS_E_INTERNAL, "unknown exception");
    }
}

extern "C" int bicos_match_bands_device(const int* devices, int ndev, const void* const* stack0,
                                        const void* const* stack1, const int* band_rows,
                                        const size_t* row_pitch, const size_t* plane_pitch,
                                        int n, int cols, int depth, const BicosConfig* cfg,
                                        int has_nxcorr, void* disparity, void* corrmap) {
    if (!cfg) return fail(BICOS_E_ARG, "null config");
    if (n < 2) return fail(BICOS_E_ARG, "need at least two images");
    if (depth != 1 && depth != 2) return fail(BICOS_E_ARG, "bad input depth");
    if (cols < 0) return fail(BICOS_E_ARG, "negative image size");
    if (!stack0 || !stack1 || !band_rows || !row_pitch || !plane_pitch)
        return fail(BICOS_E_ARG, "null band array");
    try {
        int rc = check_devices(devices, ndev);
        if (rc) return rc;
        long rows = 0;
        for (int b = 0; b < ndev; ++b) {
            if (band_rows[b] < 0) return fail(BICOS_E_ARG, "negative band height");
            rows += band_rows[b];
        }
        if (rows > 0 && cols > 0 && !disparity) return fail(BICOS_E_ARG, "null output");
        const int root = devices[0];
        const size_t dsz = has_nxcorr ? 4 : 2, csz = cfg->precision ? 8 : 4;
        const float thr = nxc_threshold(*cfg);

        // one engine per distinct device, locked for the whole call (in device order)
        std::map<int, bicos_engine*> engines;
        for (int b = 0; b < ndev; ++b) {
            if (engines.count(devices[b])) continue;
            bicos_engine* e = default_engine(devices[b]);
            if (!e) return BICOS_E_HIP;  // bicos_last_error says why
            engines[devices[b]] = e;
        }
        std::vector<std::unique_lock<std::mutex>> locks;
        for (auto& kv : engines) locks.emplace_back(kv.second->lock);

        int cur = 0;
        (void)hipGetDevice(&cur);
        // band 0 (on the root) writes straight into the maps; every other band's maps go to
        // its engine's stage and are peer-copied (a band placed on the root again -- devices
        // may repeat -- takes the same path with a device-local copy)
        // stage layout per device: the same offsets the enqueue loop below takes
        // (band_stage_offsets), so the reservation covers the last byte written
        std::map<int, size_t> stage_need;
        std::map<int, int> copies;  // bands per device (host-staged copies: one event each)
        for (int b = 1; b < ndev; ++b) {
            size_t sd = 0, sc = 0;
            band_stage_offsets(stage_need[devices[b]], band_rows[b], cols, dsz, corrmap ? csz : 0,
                               &sd, &sc);
            ++copies[devices[b]];
        }
        // per device: true = direct peer DMA into the root's maps (or a device-local copy on
        // the root itself), false = through pinned host memory (enable_peer_path refused).
        // UNVERIFIED on distinct GPUs until a multi-GPU box runs tests/test_multi_gpu.py.
        // BICOS_GATHER_HOST=1 takes the host-staged path everywhere (read per call: the
        // one-GPU test of that path, tests/test_multi_gpu.py)
        const bool force_host = std::getenv("BICOS_GATHER_HOST") != nullptr;
        std::map<int, bool> direct;
        for (auto& kv : stage_need) {
            bicos_engine* e = engines[kv.first];
            rc = reserve(e->stage, e->stage_bytes, kv.second, e->device, e->own_stream, e->ws_ready);
            if (!rc) rc = check_hip(hipSetDevice(e->device), "hipSetDevice");
            if (!rc) rc = check_hip(hipStreamWaitEvent(e->own_stream, e->ws_ready, 0), "hipStreamWaitEvent");
            direct[e->device] = !force_host && (e->device == root || (!rc && enable_peer_path(e->device, root)));
            if (!rc && !direct[e->device]) {
                // the host-staged gather: the stage layout mirrored in this engine's pinned
                // buffer, one event per band for the root's stream to wait on
                if (e->gather_pinned_bytes < kv.second) {
                    if (e->gather_pinned) (void)hipHostFree(e->gather_pinned);
                    e->gather_pinned = nullptr;
                    e->gather_pinned_bytes = 0;
                    rc = check_hip(hipHostMalloc(&e->gather_pinned, kv.second, hipHostMallocDefault),
                                   "hipHostMalloc(gather staging)");
                    if (!rc) e->gather_pinned_bytes = kv.second;
                }
                while (!rc && (int)e->gather_events.size() < copies[e->device]) {
                    hipEvent_t ev;
                    rc = check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
                    if (!rc) e->gather_events.push_back(ev);
                }
            }
            if (rc) {
                (void)hipSetDevice(cur);
                return rc;
            }
        }
        bicos_engine* re = engines[root];
        std::map<int, int> ev_used;
        // enqueue every band (asynchronous per device), then drain
        std::map<int, size_t> used;
        long r0 = 0;
        for (int b = 0; b < ndev && rc == BICOS_OK; ++b) {
            const int br = band_rows[b];
            bicos_engine* e = engines[devices[b]];
            char* dst_d = disparity ? (char*)disparity + (size_t)r0 * cols * dsz : nullptr;
            char* dst_c = corrmap ? (char*)corrmap + (size_t)r0 * cols * csz : nullptr;
            r0 += br;
            if (br == 0 || cols == 0) continue;
            if (!stack0[b] || !stack1[b]) {
                rc = fail(BICOS_E_ARG, "null band stack");
                break;
            }
            rc = check_hip(hipSetDevice(e->device), "hipSetDevice");
            if (rc) break;
            if (b == 0) {
                rc = match_device(e, stack0[b], stack1[b], n, br, cols, row_pitch[b], plane_pitch[b],
                                  depth, *cfg, has_nxcorr != 0, thr, dst_d, dst_c, e->own_stream);
                continue;
            }
            size_t od = 0, oc = 0;
            band_stage_offsets(used[devices[b]], br, cols, dsz, corrmap ? csz : 0, &od, &oc);
            char* sd = (char*)e->stage + od;
            char* sc = corrmap ? (char*)e->stage + oc : nullptr;
            rc = match_device(e, stack0[b], stack1[b], n, br, cols, row_pitch[b], plane_pitch[b],
                              depth, *cfg, has_nxcorr != 0, thr, sd, sc, e->own_stream);
            const size_t bd = (size_t)br * cols * dsz, bc = (size_t)br * cols * csz;
            if (direct[e->device]) {
                if (!rc)
                    rc = check_hip(hipMemcpyPeerAsync(dst_d, root, sd, e->device, bd, e->own_stream),
                                   "gather (peer copy)");
                if (!rc && corrmap)
                    rc = check_hip(hipMemcpyPeerAsync(dst_c, root, sc, e->device, bc, e->own_stream),
                                   "gather (peer copy)");
                continue;
            }
            // host-staged: down on the band's stream, up on the root's once that is done
            char* hd = (char*)e->gather_pinned + od;
            char* hc = corrmap ? (char*)e->gather_pinned + oc : nullptr;
            hipEvent_t ev = e->gather_events[ev_used[e->device]++];
            if (!rc) rc = check_hip(hipMemcpyAsync(hd, sd, bd, hipMemcpyDeviceToHost, e->own_stream), "gather (download)");
            if (!rc && corrmap)
                rc = check_hip(hipMemcpyAsync(hc, sc, bc, hipMemcpyDeviceToHost, e->own_stream), "gather (download)");
            if (!rc) rc = check_hip(hipEventRecord(ev, e->own_stream), "hipEventRecord");
            if (!rc) rc = check_hip(hipSetDevice(root), "hipSetDevice");
            if (!rc) rc = check_hip(hipStreamWaitEvent(re->own_stream, ev, 0), "hipStreamWaitEvent");
            if (!rc) rc = check_hip(hipMemcpyAsync(dst_d, hd, bd, hipMemcpyHostToDevice, re->own_stream), "gather (upload)");
            if (!rc && corrmap)
                rc = check_hip(hipMemcpyAsync(dst_c, hc, bc, hipMemcpyHostToDevice, re->own_stream), "gather (upload)");
        }
        // drain every engine's stream whatever happened; the stage is reused next call
        for (auto& kv : engines) {
            bicos_engine* e = kv.second;
            (void)hipSetDevice(e->device);
            (void)hipEventRecord(e->ws_ready, e->own_stream);
            const int r = check_hip(hipStreamSynchronize(e->own_stream), "hipStreamSynchronize");
            if (!rc) rc = r;
        }
        (void)hipSetDevice(cur);
        return rc;
    } catch (const std::exception& ex) {
        return fail(BICOS_E_INTERNAL, ex.what());
    } catch (...) {
        return fail(BICOS_E_INTERNAL, "unknown exception");
    }
}
