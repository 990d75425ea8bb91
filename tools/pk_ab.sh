# A/B of search library builds (LIBS: build/<name>.so; "cur" = the working tree's) on one
# config, each run also timing variant 65 (one-product keys) in the same process
set -o pipefail
mkdir -p gpurun_out
cp libbicos_amd/libbicos_amd.so build/cur.so
for c in ${SCS:-cfg2}; do
for l in ${LIBS:-cur}; do
  cp build/$l.so libbicos_amd/libbicos_amd.so
  timeout -k 10 200 python tools/search_sweep.py --config $c --variants ${VARS:-0:0:0,65:4:8} --rounds ${ROUNDS:-3} ${RND:+--random} > gpurun_out/pkab_${c}_${l}.txt 2>&1 || { cp build/cur.so libbicos_amd/libbicos_amd.so; cat gpurun_out/pkab_${c}_${l}.txt; exit 1; }
  echo "== $c $l"; grep '"ms_median"' gpurun_out/pkab_${c}_${l}.txt | sed 's/.*"variant": \([0-9]*\).*"ms_median": \([0-9.]*\).*/v\1 \2/'
done; done
cp build/cur.so libbicos_amd/libbicos_amd.so
