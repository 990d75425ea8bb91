set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "pk_search or full_frame" > gpurun_out/pk_tests.txt 2>&1 || { tail -30 gpurun_out/pk_tests.txt; exit 1; }
tail -2 gpurun_out/pk_tests.txt
LIBS="cur" VARS=0:0:0,64:2:8,64:2:8:32,64:4:8:48,65:4:8 bash tools/pk_ab.sh || exit 1
LIBS="pkdiag1 pkdiag2" VARS=0:0:0 bash tools/pk_ab.sh
