#!/bin/bash
# Round-4 final measurement session at HEAD (one gpurun call): GPU tests, smoke, every
# BASELINE bench line, the integration grid, rocprofv3 kernel stats one frame at a time, and
# the PMC HBM-byte passes at the final kernel sources. Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/pmc gpurun_out/integ_grid.jsonl
step() { echo "=== $*"; }
step pytest
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/pytest_gpu.txt
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 \
  || { tail -20 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
step pmc
bash tools/gpu_session.sh pmchead > /dev/null || exit 1
PMCSETS="integ-n16:1 integ-n6:1 integ-n8:1 integ-n12:1" bash tools/gpu_session.sh pmchead > /dev/null || exit 1
# the bench lines below cite these bytes (same source hash); the summary comes back in gpurun_out
python tools/pmc_summary.py gpurun_out/pmc profiles/pmc_r04.json && cp profiles/pmc_r04.json gpurun_out/pmc_r04.json
step bench
bash tools/gpu_session.sh benchall > /dev/null || exit 1
for c in cfg2 cfg3 cfg4 cfg5 readme cfg1; do tail -1 gpurun_out/bench_$c.txt | cut -c1-120; done
step integ
bash tools/integ_grid.sh gpurun_out/integ_grid.jsonl || exit 1
# profiles/bench_r04.jsonl = the 6 BASELINE lines, then the 20 integration lines
for c in cfg2 cfg3 cfg4 cfg5 readme cfg1; do tail -1 gpurun_out/bench_$c.txt; done > gpurun_out/bench_r04.jsonl
cat gpurun_out/integ_grid.jsonl >> gpurun_out/bench_r04.jsonl
step profiso
SCS="cfg2 cfg3 cfg4 cfg5 cfg1 readme integ-n16 integ-n6 integ-n8 integ-n12" bash tools/gpu_session.sh profiso > /dev/null || exit 1
echo done
