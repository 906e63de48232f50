#!/bin/bash
# Interleaved A/B of two in-tree library builds on the sep kernel (config 3):
# LIBS="a.so b.so" bash scripts/ab_libs.sh.  Each round runs every library in
# its own process (scripts/ab_sep.py, layout VARIANTS, default "q").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: "${LIBS:?set LIBS}"
ROUNDS_OUT=${ROUNDS_OUT:-3}
for r in $(seq 1 $ROUNDS_OUT); do
  for L in $LIBS; do
    out=$(VIABEL_AMD_LIB=$PWD/$L VARIANTS=${VARIANTS:-q} ROUNDS=${ROUNDS:-3} STEPS=${STEPS:-4096} \
          timeout -k 10 120 python scripts/ab_sep.py 2>/dev/null | tail -1) || exit $?
    echo "$L round $r $out" | tee -a gpurun_out/ab_libs.log
  done
done
