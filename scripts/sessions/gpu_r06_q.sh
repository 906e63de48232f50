#!/bin/bash
# Round 6: block kernel update chain -- the schedule's step size and the window
# pre-sum read at the step's start, CHIVI's two columns read together, the column
# sums without selects on the add chain; block / config / IA / switch tests, then an
# interleaved A/B against the previous block kernel (libviabel_amd_base.so, the tree's
# other sources equal) on configs 1, 2 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06q
timeout -k 10 900 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_ia.py tests/test_gpu_switches.py tests/test_gpu_notebooks.py tests/test_gpu_restarts.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06q/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06q/pytest.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg1,cfg2,cfg5 ROUNDS=3 LIBS="base new" bash scripts/gpu_ab_legs.sh
