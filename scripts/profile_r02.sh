#!/bin/bash
# rocprofv3 passes for the round-2 bench line (output under gpurun_out/prof2/):
#  trace      kernel trace + stats of EXACTLY the driver's command
#             (bench.py --gpus 1 --steps 20 --warmup 5)
#  n128_*/n256_*  one PMC group per pass (never combined with trace domains) on a
#             headline-only run whose sep_kernel dispatches are 5, 256 and 20
#             steps long, so that scripts/summarize_r02.py can fit per-launch
#             models a + b * steps for HBM bytes and VALU instructions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof2
mkdir -p $OUT
PASSES=${PASSES:-"trace pmc"}
if [[ " $PASSES " == *" trace "* ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || exit $?
fi
if [[ " $PASSES " == *" pmc "* ]]; then
  for NS in 128 256; do
    ARGS="--steps 276 --warmup 5 --no-cpu-baseline --legs none --n-samples $NS"
    timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/n${NS}_fetch -o run --output-format csv -- \
      python3 bench.py $ARGS > $OUT/n${NS}_fetch.log 2>&1 || exit $?
    timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/n${NS}_write -o run --output-format csv -- \
      python3 bench.py $ARGS > $OUT/n${NS}_write.log 2>&1 || exit $?
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      -d $OUT/n${NS}_sq -o run --output-format csv -- \
      python3 bench.py $ARGS > $OUT/n${NS}_sq.log 2>&1 || exit $?
  done
fi
find $OUT -name "*.csv" | head -40
