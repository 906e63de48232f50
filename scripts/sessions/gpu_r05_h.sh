#!/bin/bash
# Round 5, GPU session h: full-rank tests; config-4 A/B (PCG on symmetric sums in
# XCD-grouped order with per-wave scalar sums vs the separate-launch PCG); phase
# stamps; symmetric-sum ubench (cold / hot operands); VALU issue costs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_switches.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_h.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for E in "VIABEL_AMD_FR_PCG_SS=0" "VIABEL_AMD_FR_PCG_SS=1"; do
    echo -n "[$E] "; env $E timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_ssprof.so timeout -k 5 120 python scripts/bench_fr.py --steps 12 \
  > gpurun_out/ss_prof_h.log 2>&1 || exit $?
python scripts/ss_phases.py gpurun_out/ss_prof_h.log | tee gpurun_out/ss_phases_h.txt
B=scripts/ubench/symsum_bench
for NS in 8 1; do
  timeout -k 5 60 $B 512 0 $NS > gpurun_out/symsum_h_$NS.log 2>&1 || exit $?
  cat gpurun_out/symsum_h_$NS.log
done
timeout -k 5 60 scripts/ubench/valu_rates > gpurun_out/valu_rates.log 2>&1 || exit $?
cat gpurun_out/valu_rates.log
