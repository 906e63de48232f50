#!/bin/bash
# Round 5, GPU session e: full-rank + switch tests on the current tree; config-4
# A/B of the PCG loops and its step timeline; host cost of the headline's launch
# pair as direct launches vs a replayed hipGraph; config-5 stage counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_switches.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_e.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_e.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for E in "VIABEL_AMD_FR_PCG_SS=0" "VIABEL_AMD_FR_PCG_SS=1"; do
    echo -n "[$E] "; env $E timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
OUT=gpurun_out/prof_fr bash scripts/gpu_cfg4_timeline.sh || exit $?
timeout -k 5 60 scripts/ubench/graph_launch > gpurun_out/graph_launch.log 2>&1 || exit $?
cat gpurun_out/graph_launch.log
bash scripts/gpu_cfg5_pmc.sh > gpurun_out/cfg5_pmc.log 2>&1 || exit $?
tail -3 gpurun_out/cfg5_pmc.log
