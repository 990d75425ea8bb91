#!/bin/bash
# Round-6 GPU sessions (one gpurun call each; every GPU step under its own time limit,
# stopping at the first crash / timeout).
#   bash tools/r06_session.sh tests     GPU tests + smoke
#   bash tools/r06_session.sh inflight  frames-in-flight A/B at N = 1 (tools/inflight_ab.sh)
#   bash tools/r06_session.sh mfma      sustained MFMA rates incl. the scaled form
set -o pipefail
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    tests)
      echo "=== pytest"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_gpu.txt 2>&1
      rc=$?; tail -15 gpurun_out/pytest_gpu.txt
      [ $rc -eq 0 ] || exit $rc
      echo "=== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 \
        || { tail -20 gpurun_out/smoke.txt; exit 1; }
      tail -1 gpurun_out/smoke.txt ;;
    inflight)
      bash tools/inflight_ab.sh || exit 1 ;;
    mfma)
      timeout -k 10 200 ./build/mfma_rate > gpurun_out/mfma_r06.txt 2>&1 || exit 1
      cat gpurun_out/mfma_r06.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
