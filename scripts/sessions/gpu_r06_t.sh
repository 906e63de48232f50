#!/bin/bash
# Round 6: host split of config 5's bounds / PSIS stage (scripts/cfg5_stage_host.py) and
# three config-5 legs of bench.py, to see where the stage's run-to-run spread comes from.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06t
timeout -k 10 300 python -u scripts/cfg5_stage_host.py > gpurun_out/r06t/stage_host.log 2>&1 || exit $?
cat gpurun_out/r06t/stage_host.log | grep '^{'
LEGS=cfg5 ROUNDS=3 LIBS="new" bash scripts/gpu_ab_legs.sh
