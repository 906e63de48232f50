#!/bin/bash
# Round-4 micro-benchmarks: GEMM phase timing (plain, symmetric, Newton-Schulz T
# epilogue) and HBM streaming-kernel variants.  Each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for a in "0 0" "1 0" "1 1" "0 1"; do
  echo "== gemm_phase sym/mode $a"; timeout -k 5 60 ./scripts/ubench/gemm_phase $a || exit $?
done > gpurun_out/gemm_phase_r04.log 2>&1
cat gpurun_out/gemm_phase_r04.log
timeout -k 5 120 ./scripts/ubench/hbm_probe > gpurun_out/hbm_probe.log 2>&1 || exit $?
cat gpurun_out/hbm_probe.log
