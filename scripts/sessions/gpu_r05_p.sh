#!/bin/bash
# Round 5, GPU session p: the flop-tally test, then the driver command under
# rocprofv3 with the library's contexts released before teardown, and the config-4
# step timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullrank.py -x -q -k "flop_tally or config4" \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_p.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_p.log
[ $rc -ne 0 ] && exit $rc
TRACE_ONLY=1 bash scripts/gpu_record_r05.sh
