#!/bin/bash
# Round-4 divergence passes with four loads in flight: bounds / PSIS / restart tests,
# then an interleaved A/B of config 5 against the previous commit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bounds_psis.py tests/test_gpu_reference_bounds.py tests/test_gpu_restarts.py tests/test_gpu_notebooks.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_r.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg5 LIBS="prev new" ROUNDS=4 bash scripts/gpu_ab_legs.sh > gpurun_out/div_unroll_ab.log 2>&1 || { cat gpurun_out/div_unroll_ab.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/div_unroll_ab.log
