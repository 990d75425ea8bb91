"""Row-band pipelining of one match across two streams (prototype on the stage entry
points): transform of band b+1 and the NXC agree of band b-1 run on a second stream while
the search of band b runs, so the HBM-bound stages can take the CU slots the compute-bound
search leaves free. Every stage is row-local, so the maps are identical.

  python tools/band_pipe_bench.py [--config cfg2] [--bands 1,2,3,4] [--rounds 5] [--reps 10]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from libbicos_amd import device  # noqa: E402
from libbicos_amd.distributed import band_rows  # noqa: E402
from libbicos_amd.synthetic import stereo_stack  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--bands", default="1,2,3,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    C = bench.CONFIGS[args.config]
    n, H, W = C["n"], C["H"], C["W"]
    cfg = device.MatchConfig(**C["cfg"])
    words = device.descriptor_words(n, cfg.mode)
    ub = device.used_bits(n, cfg.mode)
    L, R = stereo_stack(n, H, W, np.uint8)
    s0, s1 = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    eng = device.Engine(0)
    mv = None if cfg.min_variance is None else cfg.min_variance * n
    thr, step = cfg.nxcorr_threshold, cfg.subpixel_step
    sA = torch.cuda.current_stream()
    sB = torch.cuda.Stream()
    pitch = device._lib.lib().bicos_desc_pitch(W, words)

    def setup(nb):
        bands = []
        for b in range(nb):
            r0, r1 = band_rows(H, nb, b)
            bands.append(dict(
                L=s0[:, r0:r1], R=s1[:, r0:r1],
                d0=torch.empty((r1 - r0, pitch), dtype=torch.int32, device="cuda"),
                d1=torch.empty((r1 - r0, pitch), dtype=torch.int32, device="cuda"),
                raw=torch.empty((r1 - r0, W), dtype=torch.int16, device="cuda"),
                eT=torch.cuda.Event(), eS=torch.cuda.Event()))
        return bands

    def run(bands, res):
        sB.wait_stream(sA)
        for bd in bands:
            eng.transform(bd["L"], cfg.mode, words, out=bd["d0"], stream=sB)
            eng.transform(bd["R"], cfg.mode, words, out=bd["d1"], stream=sB)
            bd["eT"].record(sB)
        outs = []
        for bd in bands:
            sA.wait_event(bd["eT"])
            eng.search(bd["d0"], bd["d1"], W, words, 1, out=bd["raw"], stream=sA, bits=ub)
            bd["eS"].record(sA)
            sB.wait_event(bd["eS"])
            outs.append(eng.agree(bd["raw"], bd["L"], bd["R"], thr, mv, step, stream=sB))
        sA.wait_stream(sB)
        if res is not None:
            res.extend(outs)

    ref = None
    configs = [int(x) for x in args.bands.split(",")]
    state = {nb: setup(nb) for nb in configs}
    for nb in configs:
        res = []
        run(state[nb], res)
        torch.cuda.synchronize()
        d = torch.cat([r[0] for r in res]).cpu().numpy()
        c = torch.cat([r[1] for r in res]).cpu().numpy()
        if ref is None:
            md, mc = eng.match(s0, s1, cfg)
            ref = (md.cpu().numpy(), mc.cpu().numpy())
        if not (np.array_equal(d.view(np.uint32), ref[0].view(np.uint32)) and
                np.array_equal(c.view(np.uint32), ref[1].view(np.uint32))):
            raise SystemExit("bands=%d: maps differ from the one-call match" % nb)
    times = {nb: [] for nb in configs}
    times["match"] = []
    for _ in range(args.rounds):
        for nb in configs + ["match"]:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(sA)
            for _ in range(args.reps):
                if nb == "match":
                    eng.match(s0, s1, cfg)
                else:
                    run(state[nb], None)
            b.record(sA)
            torch.cuda.synchronize()
            times[nb].append(a.elapsed_time(b) / args.reps)
    for nb, v in times.items():
        print(json.dumps({"config": args.config, "bands": nb, "ms_median": round(statistics.median(v), 4),
                          "ms_min": round(min(v), 4)}), flush=True)


if __name__ == "__main__":
    main()
