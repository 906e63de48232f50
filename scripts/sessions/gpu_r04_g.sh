#!/bin/bash
# Round-4: block-kernel barrier timestamps at configs 1 and 2 (VB_BLOCK_TS build,
# libviabel_amd_ts.so) and the config-4 one-step timeline of the current build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_ts.so timeout -k 10 120 python -u scripts/block_phase_cfg12.py \
  > gpurun_out/block_ts.log 2>&1 || { tail -20 gpurun_out/block_ts.log; exit 1; }
grep -E "==|BLOCKTS" gpurun_out/block_ts.log | head -40
bash scripts/gpu_cfg4_timeline.sh || exit $?
