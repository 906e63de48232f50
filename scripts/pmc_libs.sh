#!/bin/bash
# SQ instruction / cycle counters of the sep kernel for several library builds:
# LIBS="a.so b.so" bash scripts/pmc_libs.sh  -> gpurun_out/pmc/<lib>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
: "${LIBS:?set LIBS}"
for L in $LIBS; do
  n=$(basename $L .so)
  VIABEL_AMD_LIB=$PWD/$L VARIANTS=q ROUNDS=1 STEPS=${STEPS:-2048} timeout -s KILL 90 \
    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS \
    -d gpurun_out/pmc/$n -o run --output-format csv -- python3 scripts/ab_sep.py > gpurun_out/pmc_$n.log 2>&1 || exit $?
done
