#!/bin/bash
# Round-4 GEMM / config-4 check: the two-pass GEMM epilogue (current build) and the
# weights hook (VIABEL_AMD_FR_WEIGHTS_FUSE=1) -- full-rank and config tests on both,
# GEMM chain old vs new header, GEMM phase stamps, config-4 A/Bs.  Each GPU step has
# its own limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_configs.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_b1.log 2>&1
rc=$?; echo "tests (default) rc=$rc"; tail -2 gpurun_out/pytest_b1.log; [ $rc -ne 0 ] && exit $rc
VIABEL_AMD_FR_WEIGHTS_FUSE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_configs.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_b2.log 2>&1
rc=$?; echo "tests (weights fused) rc=$rc"; tail -2 gpurun_out/pytest_b2.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  echo old; timeout -k 5 60 ./scripts/ubench/gemm_chain_old 512 || exit $?
  echo new; timeout -k 5 60 ./scripts/ubench/gemm_chain 512 || exit $?
done > gpurun_out/gemm_chain_ab.log 2>&1
cat gpurun_out/gemm_chain_ab.log
timeout -k 5 60 ./scripts/ubench/gemm_phase 0 0 > gpurun_out/gemm_phase_b.log 2>&1 || exit $?
timeout -k 5 60 ./scripts/ubench/gemm_phase 1 1 >> gpurun_out/gemm_phase_b.log 2>&1 || exit $?
cat gpurun_out/gemm_phase_b.log
LIBS="base new" ROUNDS=3 bash scripts/gpu_ab_fr2.sh > gpurun_out/fr_ab_epi.log 2>&1 || exit $?
cat gpurun_out/fr_ab_epi.log
ENVA="" ENVB="VIABEL_AMD_FR_WEIGHTS_FUSE=1" ROUNDS=3 bash scripts/gpu_ab_env.sh > gpurun_out/fr_ab_w.log 2>&1 || exit $?
cat gpurun_out/fr_ab_w.log
