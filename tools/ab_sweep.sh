#!/bin/bash
# A/B of several builds over the same search_sweep variants, interleaved twice, in one
# session: LIBS="cur x y" (build/<x>.so; cur = the working tree's library), SV = variants,
# SC = config. Output: gpurun_out/abs_<lib>_<k>_<cfg>.txt
set -u
mkdir -p gpurun_out build
cp libbicos_amd/libbicos_amd.so build/cur.so
for k in 1 2; do
    for l in ${LIBS}; do
        cp build/$l.so libbicos_amd/libbicos_amd.so
        timeout -k 10 300 python tools/search_sweep.py --config ${SC:-cfg2} --variants ${SV:-0:0:0} \
            > gpurun_out/abs_${l}_${k}_${SC:-cfg2}.txt 2>&1
        rc=$?
        echo "abs $l $k rc=$rc" >> gpurun_out/session.log
        if [ $rc -ne 0 ]; then cp build/cur.so libbicos_amd/libbicos_amd.so; exit $rc; fi
    done
done
cp build/cur.so libbicos_amd/libbicos_amd.so
