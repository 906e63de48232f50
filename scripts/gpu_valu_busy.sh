#!/bin/bash
# Measured VALU-busy ratio of the headline sep_kernel: one
# rocprofv3 PMC pass (SQ_ACTIVE_INST_VALU, SQ_INSTS_VALU, SQ_WAVE_CYCLES,
# SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE; no trace domains) over the driver's headline
# command, summarised by scripts/valu_busy.py into gpurun_out/valu_busy.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_valu
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $OUT -o run --output-format csv -- python3 bench.py --legs none --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 \
  > $OUT.log 2>&1 || exit $?
f=$(find $OUT -name "*counter_collection.csv" | head -1)
# the raw counters travel with the summary (RAW: the committed copy it cites)
RAW=${RAW:-gpurun_out/valu_busy_counters.csv}
cp "$f" "$RAW" || exit 1
python3 scripts/valu_busy.py "$RAW" > gpurun_out/valu_busy.json && cat gpurun_out/valu_busy.json
