#!/bin/bash
# Frames in flight at N = 1: F = FLS (default 1 2 3) interleaved per config,
# ROUNDS passes, at the driver's default step count (20) and a longer one (STEPSLIST). One JSON
# line per run in gpurun_out/inflight_r06.jsonl. Stops at the first crash / timeout.
set -u
mkdir -p gpurun_out
out=${OUT:-gpurun_out/inflight_r06.jsonl}
for r in $(seq ${ROUNDS:-2}); do
  for c in ${SCS:-cfg1 cfg2 cfg3 cfg4 cfg5}; do
    for steps in ${STEPSLIST:-20 200}; do
      for f in ${FLS:-1 2 3}; do
        timeout -k 10 120 python bench.py --config $c --inflight $f --steps $steps --warmup 3 \
            --no-cpu-baseline --no-host-path --kernel-reps 0 > gpurun_out/ifl.txt 2> gpurun_out/ifl.err
        rc=$?
        if [ $rc -ne 0 ]; then echo "STOP rc=$rc ($c F=$f)"; tail -5 gpurun_out/ifl.err; exit $rc; fi
        python - "$c" "$f" "$r" "$steps" <<'EOF' | tee -a $out
import json, sys
c, f, r, steps = sys.argv[1:]
j = json.loads([l for l in open("gpurun_out/ifl.txt") if l.startswith("{")][-1])
print(json.dumps({"config": c, "inflight": int(f), "round": int(r), "steps": int(steps),
                  "value": j["value"], "ms_per_step": j["ms_per_step"],
                  "ms_one_at_a_time": j["ms_per_match_one_at_a_time"]}))
EOF
      done
    done
  done
done
echo done
