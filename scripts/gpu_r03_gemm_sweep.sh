#!/bin/bash
# GEMM main-loop variants (k tile x LDS stages) + rocprofv3 trace of a config-4 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in scripts/ubench/gemm_glds_check_k*; do
  echo "== $b"; timeout -k 10 60 ./$b || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fr -o fr --output-format csv -- python3 scripts/bench_fr.py --steps 10 > gpurun_out/prof_fr.log 2>&1 || exit $?
f=$(find gpurun_out/prof_fr -name "*kernel_trace.csv" | head -1)
python3 scripts/fr_step_trace.py "$f" 8 > gpurun_out/fr_step_timeline.txt
tail -12 gpurun_out/fr_step_timeline.txt
