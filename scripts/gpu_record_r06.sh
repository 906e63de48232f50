#!/bin/bash
# Round-6 final GPU record of the current tree: the whole -m gpu suite, smoke(), the
# headline counter passes and the rocprofv3 kernel trace + stats of the driver command
# (scripts/profile_r02.sh, summarised in place by scripts/summarize_r02.py r06, which
# also keeps every pass's raw counter CSV under profiles/r06/raw_counters/), the
# VALU-busy pass (its raw counters to profiles/r06/valu_busy_headline_counters.csv),
# the driver's bench command, the config-4 step timeline and the headline's per-wave
# timeline (VB_SEP_PROF build, libviabel_amd_sepprof.so).  Everything is copied under
# gpurun_out/rec/.  Each GPU step has its own time limit; the first failure ends it.
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
# (the run counts when its JSON line and the stats are there)
grep -q '^{' gpurun_out/prof2/trace.log && find gpurun_out/prof2/trace -name "*kernel_stats.csv" | grep -q . || { tail -5 gpurun_out/rec/prof2.log; exit 1; }
python3 scripts/summarize_r02.py r06 > gpurun_out/rec/summarize.log 2>&1 || { tail -5 gpurun_out/rec/summarize.log; exit 1; }
mkdir -p gpurun_out/rec/r06
cp -r profiles/traffic.json profiles/r06/pmc_per_dispatch.json profiles/r06/driver_cmd_kernel_stats.csv \
  profiles/r06/driver_cmd_dispatches.csv profiles/r06/raw_counters gpurun_out/rec/r06/
RAW=profiles/r06/valu_busy_headline_counters.csv bash scripts/gpu_valu_busy.sh > gpurun_out/rec/valu_busy.log 2>&1 || exit $?
cp gpurun_out/valu_busy.json profiles/r06/valu_busy_headline.json && cp gpurun_out/valu_busy.json \
  profiles/r06/valu_busy_headline_counters.csv gpurun_out/rec/r06/
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rec/bench.log 2>&1 || exit $?
tail -c 300 gpurun_out/rec/bench.log
OUT=gpurun_out/rec/prof_fr bash scripts/gpu_cfg4_timeline.sh || exit $?
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_sepprof.so timeout -k 10 120 python -u scripts/sep_timeline.py 20 \
  > gpurun_out/rec/sep_wave_raw.log 2>&1 || exit $?
python3 scripts/sep_timeline.py --parse gpurun_out/rec/sep_wave_raw.log > gpurun_out/rec/sep_wave_timeline.txt
cat gpurun_out/rec/sep_wave_timeline.txt
