"""End-to-end host-buffer path (the reference's main use: host images in, host maps out).

  python tools/host_bench.py [--config cfg2] [--reps 5]

Times, on one GPU: pybicos.match on numpy stacks (upload + match + download, what a
reference user calls), the device-resident match alone, and the raw H2D bandwidth of the
same bytes from pageable and from pinned host memory. One JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import pybicos  # noqa: E402
from libbicos_amd import device  # noqa: E402
from libbicos_amd.synthetic import stereo_stack  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    C = bench.CONFIGS[args.config]
    n, H, W = C["n"], C["H"], C["W"]
    dt = np.uint8 if C["dtype"] == "u8" else np.uint16
    L, R = stereo_stack(n, H, W, dt)
    nbytes = L.nbytes + R.nbytes
    mc = C["cfg"]

    cfg = pybicos.Config()
    if mc.get("nxcorr_threshold") is not None:
        cfg.nxcorr_threshold = mc["nxcorr_threshold"]
    if mc.get("subpixel_step"):
        cfg.subpixel_step = mc["subpixel_step"]
    if mc.get("min_variance"):
        cfg.min_variance = mc["min_variance"]
    if mc.get("variant") == 1:
        cfg.set_consistency(max_lr_diff=mc.get("max_lr_diff", 1), no_dupes=mc.get("no_dupes", False))
    left = [L[t] for t in range(n)]
    right = [R[t] for t in range(n)]
    sep_left = [L[t].copy() for t in range(n)]   # separately allocated images
    sep_right = [R[t].copy() for t in range(n)]
    acc = {"views of one array": [], "separate images": []}
    for rep in range(args.reps + 1):  # interleaved; the first round is warm-up
        for label, imgs in (("views of one array", (left, right)),
                            ("separate images", (sep_left, sep_right))):
            t0 = time.perf_counter()
            pybicos.match(imgs[0], imgs[1], cfg)
            if rep:
                acc[label].append(time.perf_counter() - t0)
    for label, ts in acc.items():
        t = float(np.median(ts))
        print(json.dumps({"what": "pybicos.match (host in/out)", "config": args.config,
                          "images": label, "ms": round(t * 1e3, 3),
                          "ms_min": round(min(ts) * 1e3, 3), "Mpix_s": round(H * W / t / 1e6, 1),
                          "h2d_bytes": nbytes, "reps": len(ts)}), flush=True)

    eng = device.Engine(0)
    s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    mcfg = device.MatchConfig(**{k: v for k, v in mc.items()})
    t = timed(lambda: eng.match(s0, s1, mcfg), args.reps)
    print(json.dumps({"what": "device-resident match", "config": args.config, "ms": round(t * 1e3, 3),
                      "Mpix_s": round(H * W / t / 1e6, 1)}), flush=True)

    src = torch.from_numpy(np.concatenate([L.reshape(-1), R.reshape(-1)]))
    dst = torch.empty_like(src, device="cuda")
    t = timed(lambda: dst.copy_(src, non_blocking=False), args.reps)
    print(json.dumps({"what": "H2D pageable (torch copy_)", "GBps": round(nbytes / t / 1e9, 2),
                      "ms": round(t * 1e3, 3)}), flush=True)
    pin = src.pin_memory()
    t = timed(lambda: dst.copy_(pin, non_blocking=True), args.reps)
    print(json.dumps({"what": "H2D pinned (torch copy_)", "GBps": round(nbytes / t / 1e9, 2),
                      "ms": round(t * 1e3, 3)}), flush=True)
    t = timed(lambda: pin.copy_(src), args.reps)
    print(json.dumps({"what": "host memcpy pageable->pinned (1 thread)", "GBps": round(nbytes / t / 1e9, 2),
                      "ms": round(t * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
