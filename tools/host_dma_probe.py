"""How fast do pageable host buffers move over PCIe through hipMemcpyAsync, and does the
call block the host? (the host path's breakdown.) The banded host pipeline
(engine.cpp match_host) gathers the caller's images into pinned slots first; this probe
times the alternative -- the DMA straight from the caller's (pageable) images.

  python tools/host_dma_probe.py [--config cfg2] [--reps 5]

One JSON line per case: host-side enqueue time of all copies, completion time, GB/s.
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from libbicos_amd.synthetic import stereo_stack  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    C = bench.CONFIGS[args.config]
    n, H, W = C["n"], C["H"], C["W"]
    L, R = stereo_stack(n, H, W, np.uint8)
    imgs = [L[t].copy() for t in range(n)] + [R[t].copy() for t in range(n)]
    nbytes = sum(a.nbytes for a in imgs)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    out = torch.empty(H * W * 8, dtype=torch.uint8, device="cuda")
    host_out = np.empty(H * W * 8, np.uint8)
    st = torch.cuda.Stream()
    sp = st.cuda_stream
    base = dev.data_ptr()

    def h2d(parts):
        # parts: row bands per image; every band of every image, band-major
        t0 = time.perf_counter()
        off = 0
        offs = []
        for a in imgs:
            offs.append(off)
            off += a.nbytes
        rows = H // parts
        for p in range(parts):
            for a, o in zip(imgs, offs):
                b = p * rows * W
                e = a.nbytes if p == parts - 1 else (p + 1) * rows * W
                rc = hip.hipMemcpyAsync(base + o + b, a.ctypes.data + b, e - b, 1, sp)
                assert rc == 0, rc
        t1 = time.perf_counter()
        st.synchronize()
        t2 = time.perf_counter()
        return t1 - t0, t2 - t0

    def d2h():
        t0 = time.perf_counter()
        rc = hip.hipMemcpyAsync(host_out.ctypes.data, out.data_ptr(), out.numel(), 2, sp)
        assert rc == 0, rc
        t1 = time.perf_counter()
        st.synchronize()
        return t1 - t0, time.perf_counter() - t0

    for parts in (1, 2, 4, 8):
        h2d(parts)
        r = [h2d(parts) for _ in range(args.reps)]
        enq = float(np.median([x[0] for x in r]))
        tot = float(np.median([x[1] for x in r]))
        print(json.dumps({"what": "H2D pageable, %d copies (%d images x %d row bands)" % (
            len(imgs) * parts, len(imgs), parts), "bytes": nbytes, "enqueue_ms": round(enq * 1e3, 3),
            "total_ms": round(tot * 1e3, 3), "GBps": round(nbytes / tot / 1e9, 1)}), flush=True)
    d2h()
    r = [d2h() for _ in range(args.reps)]
    print(json.dumps({"what": "D2H pageable, one copy", "bytes": out.numel(),
                      "enqueue_ms": round(float(np.median([x[0] for x in r])) * 1e3, 3),
                      "total_ms": round(float(np.median([x[1] for x in r])) * 1e3, 3),
                      "GBps": round(out.numel() / float(np.median([x[1] for x in r])) / 1e9, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
