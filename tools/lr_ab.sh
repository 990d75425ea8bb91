#!/bin/bash
set -u
mkdir -p gpurun_out
out=gpurun_out/lr_ab.jsonl
for r in 1 2; do
  for v in 1 0; do
    BICOS_LR_ONE_PASS=$v timeout -k 10 240 python bench.py --config cfg4 --steps 100 --warmup 5 --no-cpu-baseline --no-host-path > gpurun_out/lr.txt 2> gpurun_out/lr.err
    rc=$?; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; tail -5 gpurun_out/lr.err; exit $rc; fi
    python - $v $r <<'PY' | tee -a $out
import json,sys
j=json.loads([l for l in open("gpurun_out/lr.txt") if l.startswith("{")][-1])
r=j["roofline"]
print(json.dumps({"one_pass":int(sys.argv[1]),"round":int(sys.argv[2]),"value":j["value"],"ms_per_step":j["ms_per_step"],
 "search_ms":r["ms_per_launch"],"frac":r["frac"],"bound":r["bound"],"plan":r.get("plan"),"agree_ms":r["hbm"]["agree_ms"],"stage_ms":r.get("stage_after_transform_ms")}))
PY
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/lrprof -o run -- python bench.py --config cfg4 --steps 50 --warmup 5 --no-cpu-baseline --no-host-path --kernel-reps 0 > gpurun_out/lrprof.txt 2>&1 || exit 1
find gpurun_out/lrprof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/lr_kernel_stats.csv
echo done
