set -e
mkdir -p gpurun_out
for r in 1 2; do for c in cfg1 cfg2; do for f in 2 3 4; do
  timeout -k 10 120 python bench.py --config $c --inflight $f --steps 20 --warmup 3 --no-cpu-baseline --no-host-path 2>/dev/null | grep '^{' | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(json.dumps({'config':'$c','inflight':$f,'round':$r,'value':j['value'],'ms_per_step':j['ms_per_step']}))" | tee -a gpurun_out/inflight.jsonl
done; done; done
