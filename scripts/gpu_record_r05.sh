#!/bin/bash
# Round-5 GPU record on the current tree: the full -m gpu suite, smoke(), the
# driver's bench command, a rocprofv3 kernel trace + stats of that same command, and
# the config-4 step timeline.  Each GPU step has its own time limit; the first
# failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${TRACE_ONLY:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -c 400 gpurun_out/bench.log
fi
rm -rf gpurun_out/prof2/trace
mkdir -p gpurun_out/prof2
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/trace -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof2/trace.log 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
# (the profiler's own teardown has segfaulted after a complete run with the CU-masked
# pre-draw streams alive: the run counts when its JSON line and the stats are there)
grep -q '^{' gpurun_out/prof2/trace.log && find gpurun_out/prof2/trace -name "*kernel_stats.csv" | grep -q . || exit 1
[ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/prof_fr bash scripts/gpu_cfg4_timeline.sh || exit $?
