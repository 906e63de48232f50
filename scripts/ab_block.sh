#!/bin/bash
# Block-kernel per-step latency (scripts/block_latency.py) for several library
# builds, alternated: LIBS="a.so b.so" bash scripts/ab_block.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: "${LIBS:?set LIBS}"
for r in $(seq 1 ${ROUNDS_OUT:-2}); do
  for L in $LIBS; do
    VIABEL_AMD_LIB=$PWD/$L BL_STEPS=${BL_STEPS:-2000} timeout -k 10 120 python scripts/block_latency.py 2>/dev/null \
      | sed "s|^|$(basename $L) r$r |" | tee -a gpurun_out/ab_block.log || exit $?
  done
done
