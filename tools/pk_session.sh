set -o pipefail
cp libbicos_amd/libbicos_amd.so build/cur.so
cp build/tf2.so libbicos_amd/libbicos_amd.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "transform or full_frame or match_bit_exact or cfg5" > gpurun_out/tf2_tests.txt 2>&1; rc=$?
cp build/cur.so libbicos_amd/libbicos_amd.so
tail -3 gpurun_out/tf2_tests.txt
[ $rc -eq 0 ] || exit 1
LIBS="cur tf2" SCS="cfg2 cfg3" bash tools/gpu_session.sh abbench || exit 1
for l in cur tf2; do cp build/$l.so libbicos_amd/libbicos_amd.so; timeout -k 10 200 python tools/ref_kernel_bench.py --stages transform > gpurun_out/tf2_refk_$l.txt 2>&1; done
cp build/cur.so libbicos_amd/libbicos_amd.so
grep -h transform gpurun_out/tf2_refk_*.txt | head -20
