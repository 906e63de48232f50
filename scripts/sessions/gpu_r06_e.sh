#!/bin/bash
# Round 6: rolled variate loop in the polar log-weight kernel -- polar / restart
# tests, then the config-5 stage counter passes (scripts/gpu_cfg5_pmc.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06e
timeout -k 10 300 python -u -m pytest tests/test_gpu_bailey.py tests/test_gpu_restarts.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06e/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06e/pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_cfg5_pmc.sh > gpurun_out/cfg5_pmc.log 2>&1 || { tail -20 gpurun_out/cfg5_pmc.log; exit 1; }
python3 scripts/summarize_cfg5_pmc.py gpurun_out/cfg5_pmc > gpurun_out/cfg5_pmc/summary.json && head -16 gpurun_out/cfg5_pmc/summary.json
