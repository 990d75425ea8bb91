set -u
export BICOS_AGREE_RPT=2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "agree or padded or cfg2_full or cfg5" > gpurun_out/ab_agree_tests.txt 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/ab_agree_tests.txt; exit 1; }
tail -3 gpurun_out/ab_agree_tests.txt
for k in 1 2; do for rpt in 1 2; do for cfg in cfg2 cfg5; do
  BICOS_AGREE_RPT=$rpt timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > gpurun_out/ab_agree_${cfg}_${rpt}_$k.txt 2>&1 || exit 1
  python - gpurun_out/ab_agree_${cfg}_${rpt}_$k.txt $rpt <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l); h=d['roofline'].get('hbm',{})
print(d['config']['workload'][:5], 'rpt', sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'], 'agree_ms', h.get('agree_ms'), 'agree_GBps', h.get('agree_GBps'))
PY
done; done; done
