# Round-end rehearsal at HEAD: GPU tests, smoke, default bench line (driver's commands)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/final_pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/final_pytest_gpu.txt
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.txt 2>&1 || { tail -20 gpurun_out/final_smoke.txt; exit 1; }
tail -2 gpurun_out/final_smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/final_bench.txt 2>&1 || { tail -20 gpurun_out/final_bench.txt; exit 1; }
tail -1 gpurun_out/final_bench.txt
