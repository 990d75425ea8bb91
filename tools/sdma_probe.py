"""Copy-engine rates on one idle MI355X (VERDICT r05 #1 context): hipMemcpyAsync device to
device of S MB, kind hipMemcpyDeviceToDeviceNoCU (1024: no blit kernel) vs
hipMemcpyDeviceToDevice (3), on 1 / 2 / 4 streams at once, GB/s of bytes copied. One GPU has no
peer, so this is the local HBM-to-HBM rate of the engines the copy-engine gather uses.

  python tools/sdma_probe.py [--out profiles/sdma_probe_r06.jsonl]
"""
import argparse
import ctypes
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    hip.hipMemcpyAsync.restype = ctypes.c_int
    out = []
    for mb in (2, 8, 16, 64):
        n = mb << 20
        src = torch.ones(n // 4, dtype=torch.int32, device="cuda")
        dst = torch.empty_like(src)
        for kind in (1024, 3):
            for ns in (1, 2, 4):
                streams = [torch.cuda.Stream() for _ in range(ns)]
                per = n // ns

                def once():
                    for i, st in enumerate(streams):
                        rc = hip.hipMemcpyAsync(dst.data_ptr() + i * per, src.data_ptr() + i * per,
                                                per, kind, st.cuda_stream)
                        assert rc == 0, rc
                for _ in range(3):
                    once()
                torch.cuda.synchronize()
                reps = 20
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for s in streams:
                    s.wait_event(e0)
                for _ in range(reps):
                    once()
                for s in streams:
                    torch.cuda.current_stream().wait_stream(s)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                rec = {"MB": mb, "kind": "DeviceToDeviceNoCU" if kind == 1024 else "DeviceToDevice",
                       "streams": ns, "ms": round(ms, 4), "GBps": round(n / (ms * 1e-3) / 1e9, 1)}
                print(json.dumps(rec), flush=True)
                out.append(rec)
    if args.out:
        with open(args.out, "a") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
