#!/bin/bash
# Round 5, GPU session af: the CHIVI copy wave computes its window and log-sigma sums after the block-max barrier (KLVI code unchanged) --
# block / config tests, then configs 1, 2 and 5 and
# the headline against the previous commit ("prev"), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_restarts.py \
  tests/test_gpu_notebooks.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_af.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_af.log
[ $rc -ne 0 ] && exit $rc
LIBS="new prev" LEGS=cfg1,cfg2,cfg5 ROUNDS=4 bash scripts/gpu_ab_legs.sh | tee gpurun_out/ab_af.log
