#!/bin/bash
# The reference integration-bench grid on one MI355X (bench/cuda.cu:297-323,397-401): FULL mode,
# nxcorr 0.9, n = 6/8/12/16 x subpixel none / 0.25 / 0.20 / 0.15 / 0.10 at 3208x2200, one
# bench.py line per point (each carries vs_published = the RTX 4090 time of that point).
#   bash tools/integ_grid.sh [out.jsonl] [n ...]
set -o pipefail
mkdir -p gpurun_out
OUT=${1:-gpurun_out/integ_grid.jsonl}
shift || true
NS=${*:-6 8 12 16}
for n in $NS; do
  for s in "" -s25 -s20 -s15 -s10; do
    c=integ-n$n$s
    timeout -k 10 300 python bench.py --config $c --no-host-path --cpu-seconds 4 \
      > gpurun_out/integ_$c.txt 2>&1 || { tail -5 gpurun_out/integ_$c.txt; exit 1; }
    tail -1 gpurun_out/integ_$c.txt >> "$OUT"
    python - "$c" gpurun_out/integ_$c.txt <<'EOF'
import json, sys
l = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
p = l["vs_published"]
print("%-14s %8.1f Mpix/s  one-at-a-time %.3f ms  RTX4090 %.2f ms  x%.1f  search frac %.3f" % (
    sys.argv[1], l["value"], p["ours_ms_one_at_a_time"], p["ms_per_match"], p["speedup"],
    l["roofline"]["frac"]), flush=True)
EOF
  done
done
