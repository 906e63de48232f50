#!/bin/bash
# Round-4 config-5 log weights: one gamma loop per row (current build) against the
# per-pair loops (libviabel_amd_pairloops.so): log-weight / config-5 tests, then an
# interleaved A/B of the config-5 leg.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_bounds_psis.py tests/test_gpu_restarts.py \
  tests/test_gpu_notebooks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_c.log; [ $rc -ne 0 ] && exit $rc
LIBS="pairloops new" ROUNDS=3 bash scripts/gpu_ab_cfg5.sh 2>&1 | tee gpurun_out/cfg5_ab.log
