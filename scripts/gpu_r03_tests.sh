#!/bin/bash
# Round-3 GPU check: the new configuration / namespace / fallback tests first,
# then the whole GPU suite.  Each step under its own time limit; stop at the
# first crash / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SEL=${SEL:-"tests/test_gpu_configs.py tests/test_gpu_reference_bounds.py tests/test_gpu_restarts.py"}
timeout -k 10 ${T1:-600} python -u -m pytest $SEL -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_new.log 2>&1
rc=$?
echo "new tests rc=$rc"; tail -25 gpurun_out/pytest_new.log
if [ $rc -ge 2 ] || [ "${FULL:-1}" = "0" ]; then exit $rc; fi
timeout -k 10 ${T2:-600} python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc2=$?
echo "full suite rc=$rc2"; tail -15 gpurun_out/pytest_gpu.log
exit $(( rc > rc2 ? rc : rc2 ))
