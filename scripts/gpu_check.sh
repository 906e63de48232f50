#!/bin/bash
# GPU-box check: parity tests, then a short bench, then a rocprofv3 kernel
# trace of the bench.  Every GPU step has its own time limit; a crash, abort
# or timeout (exit >= 2 from pytest, any failure elsewhere) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTEST_ARGS=${PYTEST_ARGS:-"-q -m gpu"}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"; tail -5 gpurun_out/bench.log
exit $(( rc > rc2 ? rc : rc2 ))
