#!/bin/bash
# Compacted reverse search block order A/B (round 5): the random-search inputs at 128 bits with
# libraries built with different -DBICOS_REV_AHEAD / -DBICOS_REV_AHEAD_CHUNK (build/rev_*.so,
# tools/build_variant.sh), interleaved twice on one box. The working tree's library is "cur".
set -o pipefail
mkdir -p gpurun_out
cp libbicos_amd/libbicos_amd.so build/cur.so
rc=0
for k in 1 2; do
    for l in cur ${LIBS:-rev_64_0 rev_0_0 rev_32_0}; do
        cp build/$l.so libbicos_amd/libbicos_amd.so
        echo "=== $l $k"
        timeout -k 10 300 python tools/random_search_bench.py --words 4 --out gpurun_out/ro_${l}_$k.jsonl > gpurun_out/ro_${l}_$k.txt 2>&1 || { rc=$?; echo "rc=$rc"; break 2; }
    done
done
cp build/cur.so libbicos_amd/libbicos_amd.so
exit $rc
