#!/bin/bash
# Round-4: exact-epilogue bitwise test, and a rocprofv3 kernel trace of config 5's
# bounds stage (scripts/cfg5_stage_host.py) for the per-kernel split of the new PSIS path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py -k "exact_epilogue" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_o.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_o.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof_stage
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stage -o st --output-format csv -- \
  python3 scripts/cfg5_stage_host.py > gpurun_out/prof_stage.log 2>&1 || { tail -5 gpurun_out/prof_stage.log; exit 1; }
f=$(find gpurun_out/prof_stage -name "*kernel_stats.csv" | head -1)
head -30 "$f" | cut -d, -f1-4
