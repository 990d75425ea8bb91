# A/B session for one experimental library build (build/tf2.so here; edit per experiment):
# parity subset on the experimental build, whole-frame benches interleaved with the
# working tree's library (tools/gpu_session.sh abbench), reference kernel-bench shapes.
# Round 3 used it for the packed-key search, the full-first reduction and the two-pixel
# transform (profiles/pk_keys_r03.jsonl, fullfirst_r03.jsonl, transform_2px_r03.jsonl).
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
