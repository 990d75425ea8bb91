#!/bin/bash
# Round-6 final measurement session at HEAD, in two gpurun calls (each under the 20-minute
# limit). Stops at the first failing step.
#   bash tools/final_r06.sh A   GPU tests, smoke, PMC HBM bytes at the final sources, the
#                               BASELINE bench lines (cfg2 with the CPU baseline + host path)
#   bash tools/final_r06.sh B   the reference integration grid, rocprofv3 kernel stats one
#                               frame at a time, the reference kernel-bench shapes and the
#                               random-descriptor search points (32/64/128-bit)
set -o pipefail
mkdir -p gpurun_out
step() { echo "=== $*"; }
case ${1:-A} in
A)
    rm -rf gpurun_out/pmc
    step pytest
    timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
    tail -1 gpurun_out/pytest_gpu.txt
    step smoke
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 \
      || { tail -20 gpurun_out/smoke.txt; exit 1; }
    tail -1 gpurun_out/smoke.txt
    step pmc
    bash tools/gpu_session.sh pmchead > /dev/null || exit 1
    PMCSETS="integ-n16:1 integ-n6:1 integ-n8:1 integ-n12:1" bash tools/gpu_session.sh pmchead > /dev/null || exit 1
    python tools/pmc_summary.py gpurun_out/pmc profiles/pmc_r06.json && cp profiles/pmc_r06.json gpurun_out/pmc_r06.json
    step bench
    bash tools/gpu_session.sh benchall > /dev/null || exit 1
    for c in cfg2 cfg3 cfg4 cfg5 readme cfg1; do tail -1 gpurun_out/bench_$c.txt; done > gpurun_out/bench_r06.jsonl
    for c in cfg2 cfg3 cfg4 cfg5 readme cfg1; do tail -1 gpurun_out/bench_$c.txt | cut -c1-120; done
    ;;
B)
    rm -f gpurun_out/integ_grid.jsonl
    step integ
    bash tools/integ_grid.sh gpurun_out/integ_grid.jsonl || exit 1
    step profiso
    SCS="cfg2 cfg3 cfg4 cfg5 cfg1 readme integ-n16 integ-n6 integ-n8 integ-n12" bash tools/gpu_session.sh profiso > /dev/null || exit 1
    step refk
    timeout -k 10 300 python tools/ref_kernel_bench.py --out gpurun_out/ref_kernel_bench_r06.jsonl > gpurun_out/refk.txt 2>&1 || exit 1
    step random
    timeout -k 10 300 python tools/random_search_bench.py --words 1,2,4 --out gpurun_out/random_search_r06.jsonl > gpurun_out/random.txt 2>&1 || exit 1
    ;;
esac
echo done
