#!/bin/bash
# Round 6: config 5's bounds stage -- the t-family log-weight rows' log q as one log of
# the product of (1 + T^2 / df) (new) vs the sum of log1p (base = the previous commit's
# vb_mf.hip), and the PSIS k-hats on the worker thread vs after the bound algebra
# (VIABEL_AMD_PSIS_WORKER=0); Bailey / config-5 / restart tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06u
timeout -k 10 900 python -u -m pytest tests/test_gpu_bailey.py tests/test_gpu_configs.py tests/test_gpu_restarts.py tests/test_gpu_bounds_psis.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06u/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06u/pytest.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg5 ROUNDS=3 LIBS="base new new+VIABEL_AMD_PSIS_WORKER=0" bash scripts/gpu_ab_legs.sh
