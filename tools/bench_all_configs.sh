set -o pipefail
mkdir -p gpurun_out
for c in cfg2 cfg1 cfg3 cfg4 cfg5 readme; do
  timeout -k 10 400 python bench.py --config $c --no-host-path > gpurun_out/allcfg_$c.txt 2>&1 || { tail -5 gpurun_out/allcfg_$c.txt; exit 1; }
  tail -1 gpurun_out/allcfg_$c.txt | cut -c1-200
done
