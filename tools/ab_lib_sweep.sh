#!/bin/bash
# A/B library builds (build/<name>.so) x search geometries on configs, interleaved twice in one
# session:  LIBS="head alt" SCS="integ-n16 cfg2" SV="0:0:0,64:2:4:32" bash tools/ab_lib_sweep.sh
set -o pipefail
mkdir -p gpurun_out
cp libbicos_amd/libbicos_amd.so build/cur.so
for k in 1 2; do
for c in ${SCS:-cfg2}; do
for spec in ${LIBS:-cur head}; do
  # a lib may carry one environment setting: name:VAR=value
  l=${spec%%:*}; ev=; [ "$spec" != "$l" ] && ev=${spec#*:}
  cp build/$l.so libbicos_amd/libbicos_amd.so
  env $ev timeout -k 10 240 python tools/search_sweep.py --config $c --variants ${SV:-0:0:0} --rounds ${ROUNDS:-3} \
    ${RND:+--random} > gpurun_out/abl_${c}_${spec//[:=]/_}_${k}.txt 2>&1 || { cp build/cur.so libbicos_amd/libbicos_amd.so; cat gpurun_out/abl_${c}_${spec//[:=]/_}_${k}.txt; exit 1; }
  sed "s/^/$spec /" gpurun_out/abl_${c}_${spec//[:=]/_}_${k}.txt
done; done; done
cp build/cur.so libbicos_amd/libbicos_amd.so
