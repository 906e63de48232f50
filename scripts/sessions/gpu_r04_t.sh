#!/bin/bash
# Round-4 block-kernel adagrad update with the refined rsqrt: every gpu test, then an
# interleaved A/B of configs 1, 2 and 5 against the previous commit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_t.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg1,cfg2,cfg5 LIBS="prev new" ROUNDS=3 bash scripts/gpu_ab_legs.sh > gpurun_out/block_invn_ab.log 2>&1 || { cat gpurun_out/block_invn_ab.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/block_invn_ab.log
