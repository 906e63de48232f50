#!/bin/bash
# Round-4 split-row target chains (table-free log1p / reciprocals): block-kernel
# parity tests, then an interleaved A/B of configs 1, 2 and 5 against the previous commit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_notebooks.py tests/test_gpu_restarts.py tests/test_gpu_bounds_psis.py tests/test_gpu_reference_bounds.py tests/test_gpu_wide.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_q.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg1,cfg2,cfg5 LIBS="prev new" ROUNDS=3 bash scripts/gpu_ab_legs.sh > gpurun_out/mixture_chain_ab.log 2>&1 || { cat gpurun_out/mixture_chain_ab.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/mixture_chain_ab.log
