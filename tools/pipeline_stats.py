"""Per-kernel durations inside the frame pipeline, from a rocprofv3 kernel trace.

The bench's live kernel timings (roofline.hbm, roofline.ms_per_launch) launch one kernel
back to back; inside a frame the transform and agree read stacks that the 256 MB
last-level cache no longer holds. This reads `run_kernel_trace.csv` of a
`bench.py --inflight 1` run (tools/gpu_session.sh profiso) and prints, per libbicos kernel,
the median duration over the frames (launches of the back-to-back timing phase, runs of >= 3
of one kernel, are left out), and the median gap before each kernel (the previous kernel's end to its start).
"""
import csv
import json
import statistics
import sys


def short(name):
    return name.split("(anonymous namespace)::")[-1].split("(")[0]


def main(trace, config):
    rows = [r for r in csv.DictReader(open(trace)) if "bicos" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
           for r in rows]
    # runs of one kernel: the back-to-back timing phase repeats a kernel >= 3 times; a frame
    # launches each kernel once (the Consistency search twice: forward, reverse)
    runs, i = [], 0
    while i < len(seq):
        j = i
        while j + 1 < len(seq) and seq[j + 1][0] == seq[i][0]:
            j += 1
        runs.append((i, j))
        i = j + 1
    in_frame, gaps = {}, {}
    for a, b in runs:
        if b - a >= 2:
            continue
        for i in range(a, b + 1):
            k, s, e = seq[i]
            in_frame.setdefault(k, []).append((e - s) / 1e3)
            if i:
                gaps.setdefault(k, []).append((s - seq[i - 1][2]) / 1e3)
    out = {"config": config, "source": "rocprofv3 --kernel-trace, bench.py --inflight 1",
           "kernels_us_median": {k: round(statistics.median(v), 1) for k, v in in_frame.items()},
           "launches": {k: len(v) for k, v in in_frame.items()},
           "gap_before_us_median": {k: round(statistics.median(v), 1) for k, v in gaps.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
