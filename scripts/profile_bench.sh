#!/bin/bash
# rocprofv3 passes over a shortened bench run (kernel trace + stats, then one
# PMC group per pass; never combined with trace domains).  Output under
# gpurun_out/prof/<pass>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${ARGS:-"--steps 5120 --warmup 512 --no-cpu-baseline"}
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/sq -o run --output-format csv -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -20
