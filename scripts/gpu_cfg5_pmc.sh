#!/bin/bash
# Config 5 bounds / PSIS stage: kernel trace (durations) + SQ and TCC counter
# passes, each its own rocprofv3 run (gpurun_out/cfg5_pmc/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/cfg5_pmc
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 scripts/cfg5_bounds_stage.py > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS \
  -d $OUT/sq -o run --output-format csv -- python3 scripts/cfg5_bounds_stage.py > $OUT/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
  python3 scripts/cfg5_bounds_stage.py > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
  python3 scripts/cfg5_bounds_stage.py > $OUT/write.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -20
