# A/B search builds on configs: LIBS, SCS; interleaved twice
set -o pipefail
mkdir -p gpurun_out
cp libbicos_amd/libbicos_amd.so build/cur.so
for k in 1 2; do
for c in ${SCS:-cfg2}; do
for l in ${LIBS:-cur head}; do
  cp build/$l.so libbicos_amd/libbicos_amd.so
  timeout -k 10 200 python tools/search_sweep.py --config $c --variants 0:0:0 --rounds 5 ${RND:+--random} > gpurun_out/ab_${c}_${l}_${k}.txt 2>&1 || { cp build/cur.so libbicos_amd/libbicos_amd.so; exit 1; }
done; done; done
cp build/cur.so libbicos_amd/libbicos_amd.so
