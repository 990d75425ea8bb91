"""Predicted 1 -> N GPU throughput of bench.py (strong scaling, row bands + one gather per
step), for the driver's SCALE run to check. Inputs are measurements on
one MI355X, read from profiles/:

  * the band time t(N): one process matching band 0 of an N-way split with 3 frames in
    flight, nothing else on the GPU (bench.py --band-of N --inflight 3;
    profiles/root_gather_r05.jsonl rows with root_load "none");
  * rank 0's slowdown while it receives the other bands (the same band with the ingress
    written into a root buffer per step: root_load "proxy16" -- an RCCL-shaped receive of 16
    copy workgroups with the gather's back pressure -- for the RCCL gather, root_load "dma"
    for the copy-engine gather, whose receive does not run on rank 0's CUs);
  * the link: rank r's packed band (rows x W x 6 B without subpixel) crosses its own xGMI link
    to rank 0 (links in parallel); LINK_GBPS per direction, the SURVEY s8(e) assumption
    (~153 GB/s per link) and a conservative 64 GB/s beside it.

Per step: max(t_root, t_link) with t_root = t(N) x slowdown -- the gather of step k overlaps
the kernels of later steps -- and Mpix/s = H W / step.

  python tools/scale_model.py [--profile profiles/root_gather_r05.jsonl]
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = {"cfg2": (1536, 2048, 6), "cfg5": (2160, 3840, 6)}  # rows, cols, bytes/px gathered
LINK_GBPS = (153.0, 64.0)


def load(path, with_ingress=False):
    """{(config, N, root_load): median ms_per_step}; with_ingress: also {key: (all steps
    landed, median achieved ingress GB/s)} from round-6 records (tools/jl.py lines, whose
    `ingress` holds bench.py's root_load object)."""
    rows = [json.loads(l) for l in open(path) if l.strip()]
    tab, ing = {}, {}
    for r in rows:
        key = (r["config"], int(r["band_of"]), r["root_load"])
        tab.setdefault(key, []).append(r["ms_per_step"])
        g = r.get("ingress")
        if g:
            ing.setdefault(key, []).append((g["loads_issued"] == r.get("steps", g["loads_issued"]) and
                                            not g.get("steps_skipped"), g["ingress_GBps"]))
    med = {k: sorted(v)[len(v) // 2] for k, v in tab.items()}
    if not with_ingress:
        return med
    return med, {k: (all(a for a, _ in v), sorted(b for _, b in v)[len(v) // 2])
                 for k, v in ing.items()}


def dma_mode(tab, cfg, N):
    """The copy-engine rehearsal row for an N-way run: streams = the N - 1 senders' copies,
    at most 4 (round 6 rows dma1 / dma2 / dma4), else round 5's single "dma" row."""
    k = 1 if N <= 2 else 2 if N <= 4 else 4
    for m in ("dma%d" % k, "dma"):
        if (cfg, N, m) in tab:
            return m
    return "dma%d" % k


def predict(tab, n1, ingress=None):
    out = []
    for (cfg, N, mode), t in sorted(tab.items()):
        if mode != "none" or cfg not in SHAPES:
            continue
        H, W, bpp = SHAPES[cfg]
        band_bytes = -(-H // N) * W * bpp
        for gather, load_mode in (("rccl", "proxy16"), ("dma", dma_mode(tab, cfg, N))):
            tl = tab.get((cfg, N, load_mode))
            slow = (tl / t) if tl else None
            status = None
            if ingress is not None and (cfg, N, load_mode) in ingress:
                # a row counts only if every step landed its bytes and the
                # ingress mechanism itself could carry the rate the band alone needs. The
                # RCCL-shaped receive (16 copy workgroups) is far from its own copy rate: its
                # slowdown is the sharing of rank 0's CUs. The copy-engine rows are different:
                # one GPU's engines copying HBM to HBM are their own bound (the loaded step is
                # the copy time, and more streams copy slower), so below the needed rate they
                # measure the engines, not rank 0's interference -- "unrehearsed".
                landed, gbps = ingress[(cfg, N, load_mode)]
                need = (N - 1) * band_bytes / (t * 1e-3) / 1e9
                if not landed:
                    status = "unrehearsed: steps skipped"
                elif load_mode.startswith("dma") and gbps < 0.95 * need:
                    status = ("unrehearsed: one GPU's copy engines reach %.0f of the %.0f GB/s the "
                              "band alone needs (the N-GPU gather spreads it over %d senders' "
                              "engines, %.0f GB/s each)" % (gbps, need, N - 1, need / (N - 1)))
                else:
                    status = "rehearsed"
            for link in LINK_GBPS:
                t_link = band_bytes / (link * 1e9) * 1e3
                t_root = t * (slow or 1.0)
                step = max(t_root, t_link)
                mpix = H * W / (step * 1e-3) / 1e6
                base = n1.get(cfg)
                out.append({"config": cfg, "N": N, "gather": gather, "band_ms": t,
                            "root_slowdown": round(slow, 4) if slow else None,
                            "root_slowdown_source": load_mode if slow else "not measured (1.0)",
                            "rehearsal": status,
                            "link_GBps": link, "link_ms": round(t_link, 4),
                            "predicted_ms_per_step": round(step, 4),
                            "predicted_Mpix_s": round(mpix, 0),
                            "x_vs_N1": round(mpix / base, 2) if base else None})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--profile", default=os.path.join(ROOT, "profiles", "root_gather_r06.jsonl"))
    ap.add_argument("--n1", default="cfg2=7740,cfg5=4741",
                    help="measured N = 1 Mpix/s per config (bench.py at its default frames in flight)")
    args = ap.parse_args()
    n1 = {k: float(v) for k, v in (x.split("=") for x in args.n1.split(","))}
    tab, ing = load(args.profile, with_ingress=True)
    for line in predict(tab, n1, ing):
        print(json.dumps(line))


if __name__ == "__main__":
    main()
