#!/bin/bash
# Round 6: KLVI copy wave sums the first two slots of the next step's window before the
# reduction barrier (slack while the rows run) and the rest after it -- block / config /
# IA / switch tests, interleaved A/B against the previous commit on configs 1, 2 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ae
timeout -k 10 900 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_ia.py tests/test_gpu_switches.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ae/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06ae/pytest.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg1,cfg2,cfg5 ROUNDS=3 LIBS="base new" bash scripts/gpu_ab_legs.sh
