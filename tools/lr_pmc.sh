#!/bin/bash
# PMC passes over one cfg4 bench run (the one-pass Consistency search), one counter set per run
set -u
mkdir -p gpurun_out/lrpmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/lrpmc/avail.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/lrpmc/p$i -o run --output-format csv -- python bench.py --config cfg4 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --kernel-reps 0 > gpurun_out/lrpmc/p$i.txt 2>&1
  echo "pass $i rc=$?"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lrprof -o run --output-format csv -- python bench.py --config cfg4 --steps 50 --warmup 5 --no-cpu-baseline --no-host-path --kernel-reps 0 > gpurun_out/lrprof.txt 2>&1
echo "stats rc=$?"
