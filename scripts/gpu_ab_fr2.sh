#!/bin/bash
# Config-4 A/B, interleaved over LIBS (in-tree builds; "" = the default build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in $(seq 1 ${ROUNDS:-3}); do
  for L in ${LIBS:-base new}; do
    lib=$PWD/viabel_amd/libviabel_amd_$L.so; [ "$L" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    echo -n "lib=$L "; VIABEL_AMD_LIB=$lib timeout -k 5 120 python scripts/bench_fr.py --steps ${STEPS:-40} 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
