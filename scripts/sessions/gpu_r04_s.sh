#!/bin/bash
# Round-4 exact epilogue for the NT Sigma product: full-rank tests, config-4 A/B
# against the previous commit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_configs.py -k "fullrank or config4 or cfg4 or full_rank or sigma or epilogue or newton or pcg or gemm" \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_s.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_s.log; [ $rc -ne 0 ] && exit $rc
LIBS="prev new" ROUNDS=4 bash scripts/gpu_ab_fr2.sh > gpurun_out/cfg4_nt_epi_ab.log 2>&1 || { cat gpurun_out/cfg4_nt_epi_ab.log; exit 1; }
cat gpurun_out/cfg4_nt_epi_ab.log
