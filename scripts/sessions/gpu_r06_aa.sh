#!/bin/bash
# Round 6: HOT block-kernel instances with the window pre-sum and (CHIVI) the pre-drawn
# log q as compile-time facts (their general paths drop out) -- block / config / IA /
# switch tests, interleaved A/B against the previous commit on configs 1, 2 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06aa
timeout -k 10 900 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_ia.py tests/test_gpu_switches.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06aa/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06aa/pytest.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg1,cfg2,cfg5 ROUNDS=3 LIBS="base new" bash scripts/gpu_ab_legs.sh
