#!/bin/bash
# Round-4 8-schools log weights with the table log1p: log-weight / notebook / restart
# tests, then an interleaved A/B of config 5 against the previous commit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_notebooks.py tests/test_gpu_restarts.py tests/test_gpu_vb.py -k "log_weight or logw or eight or cfg5 or config5 or notebook or restart" \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_n.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_n.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg5 LIBS="prev new" ROUNDS=4 bash scripts/gpu_ab_legs.sh > gpurun_out/logw_lp_tab_ab.log 2>&1 || { cat gpurun_out/logw_lp_tab_ab.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/logw_lp_tab_ab.log
