#!/bin/bash
# HBM bytes of the cfg4 match's kernels (one PMC pass: FETCH_SIZE, WRITE_SIZE)
set -u
mkdir -p gpurun_out/lrbytes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d gpurun_out/lrbytes -o run --output-format csv -- python bench.py --config cfg4 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --kernel-reps 0 > gpurun_out/lrbytes/log.txt 2>&1
echo "pmc rc=$?"
