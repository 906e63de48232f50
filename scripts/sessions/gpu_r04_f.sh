#!/bin/bash
# Round-4: exact-feature GEMM epilogues (VIABEL_AMD_GEMM_EPI_EXACT) and the config-5
# log-weight changes: full-rank / config / headline / bounds tests on the current
# build, config-4 A/B of the exact epilogues against the kEpiAll kernels, config-5
# A/B against the previous commit's library (libviabel_amd_prev.so), then the
# two-rank one-GPU rehearsal.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_configs.py tests/test_gpu_headline.py \
  tests/test_gpu_bounds_psis.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_f.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_f.log; [ $rc -ne 0 ] && exit $rc
ENVA="VIABEL_AMD_GEMM_EPI_EXACT=0" ENVB="VIABEL_AMD_GEMM_EPI_EXACT=1" ROUNDS=4 bash scripts/gpu_ab_env.sh \
  > gpurun_out/cfg4_epi_exact_ab.log 2>&1 || exit $?
cat gpurun_out/cfg4_epi_exact_ab.log
LIBS="prev new" ROUNDS=3 bash scripts/gpu_ab_cfg5.sh > gpurun_out/cfg5_logw_ab.log 2>&1 || exit $?
cat gpurun_out/cfg5_logw_ab.log
RANKS=2 bash scripts/gpu_rehearse_ranks.sh > gpurun_out/rehearse_2ranks_summary.log 2>&1 || exit $?
cat gpurun_out/rehearse_2ranks_summary.log
