#!/bin/bash
# Diagnostic builds of the matrix-core search (results are WRONG; timing only):
#   build/diag1.so  MFMA skeleton (products + one key per tile)
#   build/diag2.so  + the first-minimum tree, no last minimum / no branch
#   build/diag3.so  the skeleton without global loads (synthetic descriptors)
# Used by tools/gpu_session.sh diag to bound where the search kernel's time goes.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/diag
for d in 1 2 3; do
    make -C libbicos_amd/csrc -j8 BUILD=../../build/diag/o$d OUT=../../build/diag$d.so \
        FLAGS_EXTRA="-DBICOS_MX_DIAG=$d" > /dev/null
    echo "build/diag$d.so"
done
