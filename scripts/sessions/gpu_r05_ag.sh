#!/bin/bash
# Round 5, GPU session ag: KLVI window sums one step ahead in the copy wave (after the
# reduction barrier, beside the update), the block-floor skeleton following the kernel's
# placements -- the whole -m gpu suite, then configs 1, 2, 5 and the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_ag.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ag.log
[ $rc -ne 0 ] && exit $rc
LIBS="new" LEGS=cfg1,cfg2,cfg5 ROUNDS=2 bash scripts/gpu_ab_legs.sh | tee gpurun_out/ab_ag2.log
