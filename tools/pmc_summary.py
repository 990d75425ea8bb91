"""Summarise rocprofv3 outputs (kernel stats + separate --pmc passes) into one JSON.

  python tools/pmc_summary.py gpurun_out profiles/pmc_rNN.json

Groups dispatches by (kernel, grid size), averages each counter per dispatch and
applies the gfx950 corrections of /opt/skills/guides/MI355X_MICROARCH.md "HBM":
FETCH_SIZE (KB) reads half the bytes of wide (16 B/lane) coalesced streams, so
hbm_read_bytes = 2 * FETCH_SIZE * 1024. The guide calibrates that factor for 16 B/lane
loads only; here it was checked for the byte-wide buffer loads of the transform too:
2 x FETCH_SIZE equals the transform's algorithmic read bytes (n planes x pixels x 2
stacks) to 0.1 % (profiles/pmc_r01.json). WRITE_SIZE (KB) is exact for 16 B/lane stores
and matched the transform's 16 B/px descriptor stores exactly.
"""
import collections
import csv
import json
import os
import re
import sys


def load(path):
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


def main():
    src, dst = sys.argv[1], sys.argv[2]
    out = {"source": "rocprofv3 --kernel-trace --stats and separate --pmc passes", "kernels": {}}
    stats = load(os.path.join(src, "prof", "run_kernel_stats.csv"))
    out["kernel_stats"] = [{k: r[k] for k in ("Name", "Calls", "AverageNs", "Percentage")}
                           for r in stats]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in sorted(os.listdir(src)):
        for r in load(os.path.join(src, sub, "run_counter_collection.csv")):
            name = r["Kernel_Name"]
            if "bicos_hip" not in name:
                continue
            m = re.search(r"::(\w+)<([^()]*)>\(", name)
            short = "%s<%s>" % (m.group(1), m.group(2)) if m else name
            key = "%s grid=%s" % (short, r["Grid_Size"])
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key, cs in sorted(agg.items()):
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes"] = d["FETCH_SIZE"] * 1024 * 2
            d["read_correction"] = "x2 (gfx950 FETCH_SIZE half-count)"
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        out["kernels"][key] = d
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", dst, len(out["kernels"]), "kernel groups")


if __name__ == "__main__":
    main()
