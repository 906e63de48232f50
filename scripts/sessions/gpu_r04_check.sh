#!/bin/bash
# Round-4 GPU check: the new / changed tests first (verbose, so a hang names its
# test), then the whole GPU suite, smoke() and the driver's bench command.  Each
# GPU step under its own time limit; the first crash / abort / timeout ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SEL=${SEL:-"tests/test_gpu_configs.py tests/test_gpu_fullrank.py"}
timeout -k 10 ${T1:-600} python -u -m pytest $SEL -v -x --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_new.log 2>&1
rc=$?
echo "new tests rc=$rc"; tail -25 gpurun_out/pytest_new.log
[ $rc -ne 0 ] && exit $rc
if [ "${FULL:-1}" = "1" ]; then
  timeout -k 10 ${T2:-700} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "full suite rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
  tail -1 gpurun_out/smoke.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
  tail -c 400 gpurun_out/bench.log
fi
