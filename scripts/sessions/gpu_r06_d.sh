#!/bin/bash
# Round 6: config 5 bounds stage after the polar t draws -- kernel trace + SQ / FETCH /
# WRITE counter passes (scripts/gpu_cfg5_pmc.sh), summarised per kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash scripts/gpu_cfg5_pmc.sh > gpurun_out/cfg5_pmc.log 2>&1 || { tail -20 gpurun_out/cfg5_pmc.log; exit 1; }
python3 scripts/summarize_cfg5_pmc.py gpurun_out/cfg5_pmc > gpurun_out/cfg5_pmc/summary.json && head -60 gpurun_out/cfg5_pmc/summary.json
