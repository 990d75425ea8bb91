set -u
mkdir -p gpurun_out
for spec in "2 cfg2" "3 cfg3"; do
  set -- $spec
  timeout -k 10 300 python bench.py --gpus $1 --config $2 --backend gloo --steps 4 --warmup 1 --no-cpu-baseline --no-host-path --verify-gather > gpurun_out/gc_gloo_$1_$2.txt 2>&1 || { tail -30 gpurun_out/gc_gloo_$1_$2.txt; exit 1; }
  grep "verify-gather" gpurun_out/gc_gloo_$1_$2.txt
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > gpurun_out/gc_n1.txt 2>&1 || { tail -30 gpurun_out/gc_n1.txt; exit 1; }
grep '^{' gpurun_out/gc_n1.txt | cut -c1-330
