#!/bin/bash
# Round 5, GPU session g: symmetric-sum product with the XCD-grouped block order
# (cold / hot operands) and its L2 counters; VALU issue costs of the noise path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=scripts/ubench/symsum_bench
for NS in 8 1 8 1; do
  timeout -k 5 60 $B 512 0 $NS > gpurun_out/symsum_g_$NS.log 2>&1 || exit $?
  cat gpurun_out/symsum_g_$NS.log
done
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/ssg_pmc1 -o run --output-format csv -- $B \
  > gpurun_out/ssg_pmc1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ssg_pmc2 -o run --output-format csv -- $B \
  > gpurun_out/ssg_pmc2.log 2>&1 || exit $?
timeout -k 5 60 scripts/ubench/valu_rates > gpurun_out/valu_rates.log 2>&1 || exit $?
cat gpurun_out/valu_rates.log
