#!/bin/bash
# Round 6: the copy wave's window sums with every slot's LDS read issued at once (the
# same additions in order) -- block / config / IA / switch tests, interleaved A/B against
# the previous commit (libviabel_amd_base.so) on configs 1, 2 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ad
timeout -k 10 900 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_ia.py tests/test_gpu_switches.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ad/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06ad/pytest.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg1,cfg2,cfg5 ROUNDS=3 LIBS="base new" bash scripts/gpu_ab_legs.sh
