#!/bin/bash
# Round-4 config-5 bounds stage: host split of the stage, the restart tests, then
# an interleaved A/B of the PSIS / bound-algebra overlap (VIABEL_AMD_RESTART_OVERLAP).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/cfg5_stage_host.py > gpurun_out/cfg5_stage_host.log 2>&1 || { tail -5 gpurun_out/cfg5_stage_host.log; exit 1; }
grep "{" gpurun_out/cfg5_stage_host.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_restarts.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_j.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_j.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg5 LIBS="new+VIABEL_AMD_RESTART_OVERLAP=0 new" ROUNDS=4 bash scripts/gpu_ab_legs.sh > gpurun_out/cfg5_overlap_ab.log 2>&1 || { cat gpurun_out/cfg5_overlap_ab.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/cfg5_overlap_ab.log
