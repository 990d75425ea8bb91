#!/bin/bash
# Diagnostic builds of the matrix-core search (results are WRONG; timing only):
#   build/diag1.so  MFMA skeleton (products + one key per tile)
#   build/diag2.so  + the first-minimum tree, no last minimum / no branch
#   build/diag3.so  the real kernel with only the first chunk of each row expanded
#   build/diag4.so  the real kernel, last-minimum path never taken (branch kept)
#   build/diag5.so  the real kernel without the last-minimum branch
# Used by tools/gpu_session.sh diag to bound where the search kernel's time goes.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/diag
for d in ${DIAGS:-1 2 3 4 5}; do
    make -C libbicos_amd/csrc -j8 BUILD=../../build/diag/o$d OUT=../../build/diag$d.so \
        FLAGS_EXTRA="-DBICOS_MX_DIAG=$d" > /dev/null
    echo "build/diag$d.so"
done
