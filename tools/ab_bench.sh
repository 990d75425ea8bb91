set -u
cp libbicos_amd/libbicos_amd.so build/cur.so
for k in 1 2; do for l in cur alt; do
  cp build/$l.so libbicos_amd/libbicos_amd.so
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path --inflight 1 > gpurun_out/abtf_${l}_$k.txt 2>&1 || { cp build/cur.so libbicos_amd/libbicos_amd.so; exit 1; }
done; done
cp build/cur.so libbicos_amd/libbicos_amd.so
