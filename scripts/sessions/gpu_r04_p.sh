#!/bin/bash
# Round-4 PSIS fast path, unrolled passes + block-aggregated compaction: PSIS tests,
# a kernel-stats profile of config 5's bounds stage, and a config-5 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bounds_psis.py tests/test_gpu_restarts.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_p.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_p.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof_stage
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stage -o st --output-format csv -- \
  python3 scripts/cfg5_stage_host.py > gpurun_out/prof_stage.log 2>&1
f=$(find gpurun_out/prof_stage -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && grep -E "sel_|gpd|lw_|logw" "$f" | cut -d, -f1-4
LEGS=cfg5 LIBS="prev new" ROUNDS=4 bash scripts/gpu_ab_legs.sh > gpurun_out/psis_sort_barriers_ab.log 2>&1 || { cat gpurun_out/psis_sort_barriers_ab.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/psis_sort_barriers_ab.log
