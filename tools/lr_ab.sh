#!/bin/bash
# One-pass Consistency A/B on cfg4: VARIANTS (env assignments, ';'-separated per variant), ROUNDS passes
set -u
mkdir -p gpurun_out
out=${OUT:-gpurun_out/lr_ab.jsonl}
IFS=';' read -ra VS <<< "${VARIANTS:-BICOS_LR_ONE_PASS=1;BICOS_LR_ONE_PASS=0}"
for r in $(seq ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    env $v timeout -k 10 240 python bench.py --config ${CFG:-cfg4} --steps 100 --warmup 5 --no-cpu-baseline --no-host-path > gpurun_out/lr.txt 2> gpurun_out/lr.err
    rc=$?; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; tail -5 gpurun_out/lr.err; exit $rc; fi
    python - "$v" $r <<'PY' | tee -a $out
import json,sys
j=json.loads([l for l in open("gpurun_out/lr.txt") if l.startswith("{")][-1])
r=j["roofline"]
print(json.dumps({"variant":sys.argv[1],"round":int(sys.argv[2]),"config":j["config"]["workload"].split(":")[0],"value":j["value"],"ms_per_step":j["ms_per_step"],
 "search_ms":r["ms_per_launch"],"frac":r["frac"],"bound":r["bound"],"plan":r.get("plan"),"agree_ms":r["hbm"]["agree_ms"],"stage_ms":r.get("stage_after_transform_ms")}))
PY
  done
done
echo done
