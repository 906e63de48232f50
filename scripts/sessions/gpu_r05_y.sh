#!/bin/bash
# Round 5, GPU session y: exp_fast on the block / column-pair kernels' serial chains --
# the whole -m gpu suite, then the headline and configs 1, 2, 5 against the previous
# commit ("prev"), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_y.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_y.log
[ $rc -ne 0 ] && exit $rc
LIBS="new prev" LEGS=cfg1,cfg2,cfg5 ROUNDS=4 bash scripts/gpu_ab_legs.sh | tee gpurun_out/ab_y.log
