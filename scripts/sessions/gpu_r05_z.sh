#!/bin/bash
# Round 5, GPU session z: block-kernel barrier timestamps at configs 1, 2 and 5 of the
# current tree (VB_BLOCK_TS build, libviabel_amd_ts.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_ts.so timeout -k 10 120 python -u scripts/block_phase_cfg12.py \
  > gpurun_out/block_ts.log 2>&1 || { tail -20 gpurun_out/block_ts.log; exit 1; }
grep -E "==|BLOCKTS|COPYTS" gpurun_out/block_ts.log | head -60
