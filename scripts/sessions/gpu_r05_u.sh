#!/bin/bash
# Round 5, GPU session u: where the headline sep_kernel's wave cycles go -- one SQ
# pass (active / issue-stalled / parked wave cycles, VALU and LDS instructions, LDS
# bank-conflict and LDS-array cycles) and one pass of VALU / SALU / branch counts,
# over the headline-only bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/sep_sq
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  -d $OUT/p1 -o run --output-format csv -- python3 bench.py --legs none --no-cpu-baseline --steps 20 --warmup 5 \
  > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM \
  -d $OUT/p2 -o run --output-format csv -- python3 bench.py --legs none --no-cpu-baseline --steps 20 --warmup 5 \
  > $OUT/p2.log 2>&1 || exit $?
find $OUT -name "*.csv" | head
