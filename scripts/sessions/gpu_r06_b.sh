#!/bin/bash
# Round 6: the new sharded IA / R-hat tests, the teardown tests, the IA and PSIS
# suites (the PSIS flag buffer moved into the context).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ia_dist.py tests/test_gpu_teardown.py tests/test_gpu_ia.py tests/test_gpu_bounds_psis.py tests/test_gpu_restarts.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r06b/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r06b/pytest.log; exit $rc
