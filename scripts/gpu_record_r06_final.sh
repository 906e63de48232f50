#!/bin/bash
# Round-6 closing GPU record of the final tree (after scripts/gpu_record_r06.sh: the block
# kernel and config-5 stage changes that followed it): the whole -m gpu suite, smoke(),
# the config-5 bounds-stage counter passes (scripts/gpu_cfg5_pmc.sh, summarised into
# profiles/r06/cfg5/ on the box before the bench reads it) and the driver's bench
# command.  Outputs under gpurun_out/rec_final/.  Each GPU step has its own time limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rec_final/cfg5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/rec_final/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/rec_final/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rec_final/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/rec_final/smoke.log
bash scripts/gpu_cfg5_pmc.sh > gpurun_out/rec_final/cfg5_pmc.log 2>&1 || { tail -20 gpurun_out/rec_final/cfg5_pmc.log; exit 1; }
python3 scripts/summarize_cfg5_pmc.py gpurun_out/cfg5_pmc > gpurun_out/rec_final/cfg5/bounds_stage_pmc.json || exit 1
cp gpurun_out/cfg5_pmc/sq/run_counter_collection.csv gpurun_out/rec_final/cfg5/bounds_stage_sq_counters.csv
cp gpurun_out/cfg5_pmc/fetch/run_counter_collection.csv gpurun_out/rec_final/cfg5/bounds_stage_fetch_counters.csv
cp gpurun_out/cfg5_pmc/write/run_counter_collection.csv gpurun_out/rec_final/cfg5/bounds_stage_write_counters.csv
cp gpurun_out/cfg5_pmc/trace/run_kernel_stats.csv gpurun_out/rec_final/cfg5/bounds_stage_kernel_stats.csv
cp gpurun_out/rec_final/cfg5/*.json gpurun_out/rec_final/cfg5/*.csv profiles/r06/cfg5/
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rec_final/bench.log 2>&1 || exit $?
tail -c 300 gpurun_out/rec_final/bench.log
