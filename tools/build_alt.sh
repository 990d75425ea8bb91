#!/bin/bash
# Build build/alt.so from kernels.hip at git revision $1 (default HEAD) for A/B runs
# (tools/gpu_session.sh ab2|ab3|ab4); the working tree's library is rebuilt afterwards.
set -e
rev=${1:-HEAD}
cp libbicos_amd/csrc/kernels.hip /tmp/kernels.cur.hip
git show "$rev":libbicos_amd/csrc/kernels.hip > libbicos_amd/csrc/kernels.hip
make -C libbicos_amd/csrc -j8 > /dev/null
cp libbicos_amd/libbicos_amd.so build/alt.so
cp /tmp/kernels.cur.hip libbicos_amd/csrc/kernels.hip
touch libbicos_amd/csrc/kernels.hip
make -C libbicos_amd/csrc -j8 > /dev/null
echo "build/alt.so = kernels.hip@$rev"
