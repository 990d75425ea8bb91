#!/bin/bash
# A/B library builds (build/<name>.so) on whole-frame bench lines, interleaved twice in one
# session:  LIBS="cur alt" SCS="cfg2 cfg5" bash tools/ab_lib_bench.sh
set -o pipefail
mkdir -p gpurun_out
cp libbicos_amd/libbicos_amd.so build/cur.so
for k in 1 2; do
for c in ${SCS:-cfg2}; do
for spec in ${LIBS:-cur head}; do
  # a lib may carry one environment setting: name:VAR=value
  l=${spec%%:*}; ev=; [ "$spec" != "$l" ] && ev=${spec#*:}
  cp build/$l.so libbicos_amd/libbicos_amd.so
  env $ev timeout -k 10 240 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-host-path \
    > gpurun_out/abb_${c}_${spec//[:=]/_}_${k}.txt 2>&1 || { cp build/cur.so libbicos_amd/libbicos_amd.so; tail -5 gpurun_out/abb_${c}_${spec//[:=]/_}_${k}.txt; exit 1; }
  python - "$spec" "$c" gpurun_out/abb_${c}_${spec//[:=]/_}_${k}.txt <<'PY'
import json, sys
l = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
h = l["roofline"]["hbm"]
print("%-8s %-6s %8.1f Mpix/s  %.4f ms/step  one %.4f  search %.4f  tf %.4f  agree %.4f (%s)" % (
    sys.argv[1], sys.argv[2], l["value"], l["ms_per_step"], l["ms_per_match_one_at_a_time"],
    l["roofline"]["ms_per_launch"], h["transform_ms"], h["agree_ms"], h["agree_stage"]), flush=True)
PY
done; done; done
cp build/cur.so libbicos_amd/libbicos_amd.so
