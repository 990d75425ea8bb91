#!/bin/bash
# print value / ms_per_step / search / transform / agree of the ab*_{cur,alt}N bench lines in gpurun_out
for f in gpurun_out/ab*_*.txt; do
    grep -h '^{' "$f" | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); r = d['roofline']
    print('%-28s %9.1f Mpix/s %.4f ms  search %.4f  transform %.4f  agree %.4f' % ('$f'.split('/')[-1], d['value'], d['ms_per_step'], r['ms_per_launch'], r['hbm']['transform_ms'], r['hbm']['agree_ms']))"
done
