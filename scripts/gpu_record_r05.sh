#!/bin/bash
# Round-5 final GPU record of the current tree: the whole -m gpu suite, smoke(), the
# headline counter passes and the rocprofv3 kernel trace + stats of the driver command
# (scripts/profile_r02.sh, summarised in place by scripts/summarize_r02.py r05 so the
# bench below reads this tree's traffic / VALU models), the VALU-busy pass, the
# driver's bench command and the config-4 step timeline.  Everything the record
# produces is copied under gpurun_out/rec/.  Each GPU step has its own time limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rec
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/rec/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/rec/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rec/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/rec/smoke.log
rm -rf gpurun_out/prof2
PASSES="pmc trace" bash scripts/profile_r02.sh > gpurun_out/rec/prof2.log 2>&1
rc=$?
# (the profiler's teardown has segfaulted after a complete traced run: the run counts
# when its JSON line and the stats are there)
grep -q '^{' gpurun_out/prof2/trace.log && find gpurun_out/prof2/trace -name "*kernel_stats.csv" | grep -q . || { tail -5 gpurun_out/rec/prof2.log; exit 1; }
python3 scripts/summarize_r02.py r05 > gpurun_out/rec/summarize.log 2>&1 || { tail -5 gpurun_out/rec/summarize.log; exit 1; }
cp profiles/traffic.json profiles/r05/pmc_per_dispatch.json profiles/r05/driver_cmd_kernel_stats.csv \
  profiles/r05/driver_cmd_dispatches.csv gpurun_out/rec/
bash scripts/gpu_valu_busy.sh > gpurun_out/rec/valu_busy.log 2>&1 || exit $?
cp gpurun_out/valu_busy.json profiles/r05/valu_busy_headline.json && cp gpurun_out/valu_busy.json gpurun_out/rec/
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rec/bench.log 2>&1 || exit $?
tail -c 300 gpurun_out/rec/bench.log
OUT=gpurun_out/rec/prof_fr bash scripts/gpu_cfg4_timeline.sh || exit $?
