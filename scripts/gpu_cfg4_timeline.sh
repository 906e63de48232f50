#!/bin/bash
# rocprofv3 kernel trace of config-4 steps (bench_fr.py) -> one-step timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof_fr}
rm -rf $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o fr --output-format csv -- python3 scripts/bench_fr.py --steps ${STEPS:-10} > $OUT.log 2>&1 || exit $?
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 scripts/fr_step_trace.py "$f" ${STEP:-8} > $OUT.timeline.txt
tail -14 $OUT.timeline.txt
grep ms_per_step $OUT.log
