"""Stage-split frame pipeline on CU-masked streams (experiment).

The one-stream match runs transform -> search -> agree back to back: the HBM-bound
transform/agree (~0.12 ms of a cfg2 frame) and the MFMA/VALU-bound search (~0.29 ms) never
overlap, and frames in flight barely help because the search grid fills every CU. Here the
search runs on a stream whose hipExtStreamCreateWithCUMask mask holds 256 - h CUs and the
transform of frame k+1 and the agree of frame k-1 run on a stream holding the other h CUs,
so the HBM stages hide under the search. Prints one JSON line per mode (ms per frame).
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from libbicos_amd import device  # noqa: E402
from libbicos_amd.synthetic import stereo_stack  # noqa: E402

NCU = 256


def masked_stream(dev, bits):
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ctypes.c_uint32 * (NCU // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(NCU // 32), words)
    if rc != 0:
        raise RuntimeError("hipExtStreamCreateWithCUMask rc=%d" % rc)
    return torch.cuda.ExternalStream(s.value, device=dev)


def masks(h, layout):
    if h == 0:
        return list(range(NCU)), list(range(NCU))
    if layout == "lo":
        hb = list(range(h))
    else:  # evenly spread
        step = NCU // h
        hb = [i * step for i in range(h)]
    sb = [i for i in range(NCU) if i not in set(hb)]
    return sb, hb


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--hs", default="0,16,32,48")
    ap.add_argument("--layouts", default="lo,il")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, H, W = 33, 1536, 2048
    L, R = stereo_stack(n, H, W)
    s0 = torch.from_numpy(L).to(dev)
    s1 = torch.from_numpy(R).to(dev)
    cfg = device.MatchConfig(nxcorr_threshold=0.96)
    eng = device.Engine(dev)
    words = device.descriptor_words(n)
    bits = device.used_bits(n)
    ref_out, _ = eng.match(s0, s1, cfg)
    torch.cuda.synchronize()

    def wall(fn, frames):
        fn(4)
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn(frames)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3 / frames

    def match_loop(k):
        for _ in range(k):
            eng.match(s0, s1, cfg)

    # spin-up
    t = time.perf_counter()
    while time.perf_counter() - t < 0.2:
        match_loop(4)
        torch.cuda.synchronize()
    print(json.dumps({"mode": "match_one_stream", "ms": round(wall(match_loop, args.frames), 4)}),
          flush=True)

    d0 = [eng.transform(s0, words=words) for _ in range(2)]
    d1 = [eng.transform(s1, words=words) for _ in range(2)]
    raws = [torch.empty((H, W), dtype=torch.int16, device=dev) for _ in range(2)]
    last = {}

    def pipeline(S, Hs):
        def run(k):
            ev_t = [torch.cuda.Event() for _ in range(k + 1)]
            ev_s = [torch.cuda.Event() for _ in range(k)]
            eng.transform(s0, words=words, out=d0[0], stream=Hs)
            eng.transform(s1, words=words, out=d1[0], stream=Hs)
            ev_t[0].record(Hs)
            for i in range(k):
                b = i % 2
                S.wait_event(ev_t[i])
                eng.search(d0[b], d1[b], W, words, out=raws[b], stream=S, bits=bits)
                ev_s[i].record(S)
                if i + 1 < k:
                    eng.transform(s0, words=words, out=d0[1 - b], stream=Hs)
                    eng.transform(s1, words=words, out=d1[1 - b], stream=Hs)
                    ev_t[i + 1].record(Hs)
                Hs.wait_event(ev_s[i])
                with torch.cuda.stream(Hs):
                    last["out"] = eng.agree(raws[b], s0, s1, 0.96, stream=Hs)[0]
        return run

    def search_only(S):
        def run(k):
            for _ in range(k):
                eng.search(d0[0], d1[0], W, words, out=raws[0], stream=S, bits=bits)
        return run

    for h in [int(x) for x in args.hs.split(",")]:
        for layout in (args.layouts.split(",") if h else ["full"]):
            sb, hb = masks(h, layout)
            S = masked_stream(dev, sb)
            Hs = masked_stream(dev, hb)
            ms = wall(pipeline(S, Hs), args.frames)
            torch.cuda.synchronize()
            same = bool(torch.equal(last["out"], ref_out))
            sms = wall(search_only(S), 20)
            print(json.dumps({"mode": "split", "h_cus": h, "layout": layout, "ms": round(ms, 4),
                              "search_alone_ms": round(sms, 4), "equal_to_match": same}),
                  flush=True)


if __name__ == "__main__":
    main()
