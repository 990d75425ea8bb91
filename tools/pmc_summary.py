"""Summarise rocprofv3 --pmc passes (one run per counter set) into one JSON.

  python tools/pmc_summary.py gpurun_out/pmc profiles/pmc_rNN.json

Input layout (tools/gpu_session.sh `pmchead` / `pmcstall`):
  <src>/source_sha                       bench.kernel_source_hash() of the profiled tree
  <src>/<config>__b<N>__<set>/run_counter_collection.csv
      bench.py --config <config> --band-of <N> --kernel-reps 0 --inflight 1 under
      rocprofv3 --pmc <set's counters>: every dispatch is an in-frame one (no back-to-back
      kernel timing loop), of the band a rank of an N-GPU run computes (N = 1: the frame).

Groups dispatches by (config, rows, kernel template), averages each counter per dispatch
and applies the gfx950 corrections of /opt/skills/guides/MI355X_MICROARCH.md "HBM":
FETCH_SIZE (KB) counts half the bytes of wide (16 B/lane) coalesced streams, so
hbm_read_bytes = 2 * FETCH_SIZE * 1024. The guide calibrates that factor for 16 B/lane
loads only; it was checked for the byte-wide buffer loads of the transform too: 2 x
FETCH_SIZE equals the transform's algorithmic read bytes (n planes x pixels x 2 stacks) to
0.1 % (profiles/pmc_r01.json). WRITE_SIZE (KB) is exact for 16 B/lane stores.
bench.py cites these bytes as `roofline.traffic` only when `source_sha` equals the sources
it runs (bench.load_traffic).
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(path):
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


def main():
    src, dst = sys.argv[1], sys.argv[2]
    from bench import CONFIGS
    from libbicos_amd.distributed import band_rows
    sha_path = os.path.join(src, "source_sha")
    out = {"source": "rocprofv3 --pmc, one pass per counter set, bench.py --kernel-reps 0 "
                     "--inflight 1 (in-frame dispatches only)",
           "source_sha": open(sha_path).read().strip() if os.path.exists(sha_path) else None,
           "kernels": {}}
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for sub in sorted(os.listdir(src)):
        m = re.match(r"([\w-]+?)__b(\d+)__(\w+)$", sub)
        if not m:
            continue
        config, N = m.group(1), int(m.group(2))
        b, e = band_rows(CONFIGS[config]["H"], N, 0)
        rows = e - b
        for path in (os.path.join(src, sub, "run_counter_collection.csv"),):
            for r in load(path):
                name = r["Kernel_Name"]
                if "bicos_hip" not in name:
                    continue
                km = re.search(r"::(\w+)<([^()]*)>\(", name) or re.search(r"::(\w+)\(", name)
                short = ("%s<%s>" % (km.group(1), km.group(2)) if km and km.lastindex == 2
                         else (km.group(1) if km else name))
                key = "%s rows=%d :: %s grid=%s" % (config, rows, short, r["Grid_Size"])
                agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta[key] = {"config": config, "rows": rows, "band_of": N, "kernel": short,
                             "grid": int(r["Grid_Size"])}
    for key, cs in sorted(agg.items()):
        d = dict(meta[key])
        d["dispatches"] = max(len(v) for v in cs.values())
        d.update({c: sum(v) / len(v) for c, v in cs.items()})
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes"] = d["FETCH_SIZE"] * 1024 * 2
            d["read_correction"] = "x2 (gfx950 FETCH_SIZE half-count)"
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        if "SQ_WAVE_CYCLES" in d and d.get("SQ_WAVE_CYCLES"):
            wc = d["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    d[c.lower() + "_frac"] = round(d[c] / wc, 4)
        if d.get("TCP_TCC_READ_REQ_sum"):
            if "TCP_TCC_READ_REQ_LATENCY_sum" in d:
                d["l2_read_latency_cycles"] = round(d["TCP_TCC_READ_REQ_LATENCY_sum"] /
                                                    d["TCP_TCC_READ_REQ_sum"], 1)
        if d.get("TCC_HIT_sum") is not None and d.get("TCC_MISS_sum") is not None:
            tot = d["TCC_HIT_sum"] + d["TCC_MISS_sum"]
            if tot:
                d["l2_hit_rate"] = round(d["TCC_HIT_sum"] / tot, 4)
        if d.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs (8 x the kernel's cycles: the search's
            # value / 8 matches its duration at the clock it holds); TA_TA_BUSY / TD_TD_BUSY
            # are summed over their instances, one per CU
            for c in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum"):
                if c in d:
                    d[c.replace("_sum", "").lower() + "_frac_per_cu"] = round(
                        d[c] / (d["GRBM_GUI_ACTIVE"] / 8) / 256, 4)
        out["kernels"][key] = d
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", dst, len(out["kernels"]), "kernel groups, source_sha", out["source_sha"])


if __name__ == "__main__":
    main()
