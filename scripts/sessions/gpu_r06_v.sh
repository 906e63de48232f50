#!/bin/bash
# Round 6: the log-weight rows' per-block log-q constant and the serial PSIS default --
# Bailey / config-5 / restart / switch tests, then config-5 legs of bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06v
timeout -k 10 900 python -u -m pytest tests/test_gpu_bailey.py tests/test_gpu_configs.py tests/test_gpu_restarts.py tests/test_gpu_switches.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06v/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06v/pytest.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg5 ROUNDS=3 LIBS="new" bash scripts/gpu_ab_legs.sh
