#!/bin/bash
# Round-4 PSIS two-digit select: the PSIS / bounds parity tests (and the notebooks),
# then an interleaved A/B of config 5 and the k-hat leg (VIABEL_AMD_PSIS_FAST_SELECT).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bounds_psis.py tests/test_gpu_reference_bounds.py tests/test_gpu_notebooks.py tests/test_gpu_restarts.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_m.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_m.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg5,khat LIBS="new+VIABEL_AMD_PSIS_FAST_SELECT=0 new" ROUNDS=4 bash scripts/gpu_ab_legs.sh > gpurun_out/psis_select_ab.log 2>&1 || { cat gpurun_out/psis_select_ab.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/psis_select_ab.log
