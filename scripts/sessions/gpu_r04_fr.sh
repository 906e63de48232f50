#!/bin/bash
# Round-4 config-4 iteration: full-rank + config tests, then an interleaved A/B of
# an environment switch (ENVA vs ENVB) on bench_fr.py, then (TL=1) a rocprofv3
# step timeline.  Each GPU step under its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 400 python -u -m pytest ${SEL:-tests/test_gpu_fullrank.py tests/test_gpu_configs.py} -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_fr.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_fr.log; [ $rc -ne 0 ] && exit $rc
fi
ENVA=${ENVA:-} ENVB=${ENVB:-} ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab_env.sh 2>&1 | tee gpurun_out/fr_ab.log || exit $?
if [ "${TL:-1}" = "1" ]; then
  bash scripts/gpu_cfg4_timeline.sh || exit $?
fi
