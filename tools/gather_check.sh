set -u
mkdir -p gpurun_out
for spec in "2 cfg2" "5 cfg2" "2 cfg3" "3 cfg4"; do
  set -- $spec
  timeout -k 10 300 python bench.py --gpus $1 --config $2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --verify-gather > gpurun_out/gc_gloo_$1_$2.txt 2>&1 || { tail -30 gpurun_out/gc_gloo_$1_$2.txt; exit 1; }
  grep "verify-gather" gpurun_out/gc_gloo_$1_$2.txt; grep '^{' gpurun_out/gc_gloo_$1_$2.txt | cut -c1-200
done
