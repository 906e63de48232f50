#!/bin/bash
# Round-4 GEMM epilogue investigation + config-4 state: tests, phase stamps of the
# store pass run twice (I-cache / TLB warm second pass) and with the output rows
# touched before the main loop, chain timings, config-4 A/B vs the base library,
# the VALU-busy PMC pass of the headline and a config-4 step timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_configs.py tests/test_gpu_headline.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_e.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_e.log; [ $rc -ne 0 ] && exit $rc
for b in gemm_phase gemm_phase_epi2 gemm_phase_ctouch; do
  for m in "0 0" "1 1"; do
    echo "== $b $m"; timeout -k 5 60 ./scripts/ubench/$b $m || exit $?
  done
done > gpurun_out/gemm_phase_e.log 2>&1
grep -E "==|span|loop start|k0 |loop end|acc summed|epi operands|tile stored|epilogue end|pass 2" gpurun_out/gemm_phase_e.log
for i in 1 2; do
  for b in gemm_chain_old gemm_chain gemm_chain_ctouch; do
    echo "$b"; timeout -k 5 60 ./scripts/ubench/$b 512 || exit $?
  done
done > gpurun_out/gemm_chain_e.log 2>&1
cat gpurun_out/gemm_chain_e.log
LIBS="base new" ROUNDS=3 bash scripts/gpu_ab_fr2.sh > gpurun_out/fr_ab_e.log 2>&1 || exit $?
cat gpurun_out/fr_ab_e.log
bash scripts/gpu_valu_busy.sh || exit $?
bash scripts/gpu_cfg4_timeline.sh || exit $?
