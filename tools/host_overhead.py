"""Host (CPU) cost per step of the multi-GPU bench loop vs the GPU time of one band match.

At N = 8 a cfg2 band match takes ~75 us on the GPU; if issuing one step (the ctypes
match call + the async RCCL gather call) costs the host as much, the N = 8 bench is
host-bound. Measures on one GPU: (1) back-to-back match calls without sync, host time
per call; (2) GPU time per match from events; (3) host time of an async dist.gather call
(world size 1, RCCL), the other per-step call of bench.py.

  python tools/host_overhead.py [--rows 192] [--reps 200]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from libbicos_amd import device  # noqa: E402
from libbicos_amd.synthetic import stereo_stack  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--rows", type=int, default=192)
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    C = bench.CONFIGS[args.config]
    n, W = C["n"], C["W"]
    mcfg = device.MatchConfig(**C["cfg"])
    L, R = stereo_stack(n, C["H"], W, np.uint8, row_begin=0, row_end=args.rows)
    s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    eng = device.Engine(0)
    buf = torch.zeros((2, args.rows, W), dtype=torch.float32, device="cuda")
    for _ in range(20):
        eng.match(s0, s1, mcfg, out=buf[0], corrmap=buf[1])
    torch.cuda.synchronize()
    # (1) host time per call, GPU running behind
    t0 = time.perf_counter()
    for _ in range(args.reps):
        eng.match(s0, s1, mcfg, out=buf[0], corrmap=buf[1])
    host_us = (time.perf_counter() - t0) / args.reps * 1e6
    torch.cuda.synchronize()
    # (2) GPU time per match
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        eng.match(s0, s1, mcfg, out=buf[0], corrmap=buf[1])
    e1.record()
    torch.cuda.synchronize()
    gpu_us = e0.elapsed_time(e1) / args.reps * 1e3
    # (3) async gather call (RCCL, world 1)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    recv = [torch.empty_like(buf)]
    for _ in range(10):
        dist.gather(buf, recv, dst=0, async_op=True).wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    works = []
    for _ in range(args.reps):
        works.append(dist.gather(buf, recv, dst=0, async_op=True))
    gather_host_us = (time.perf_counter() - t0) / args.reps * 1e6
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print(json.dumps({"config": args.config, "band_rows": args.rows,
                      "match_host_us_per_call": round(host_us, 1),
                      "match_gpu_us": round(gpu_us, 1),
                      "gather_host_us_per_call": round(gather_host_us, 1)}), flush=True)


if __name__ == "__main__":
    main()
