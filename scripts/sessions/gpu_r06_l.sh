#!/bin/bash
# Round 6 (after CHIVI qnext): per-row-wave barrier-exit timestamps of the block kernel (VB_BLOCK_TS build,
# scripts/build_variant.sh ts) at configs 1, 2 and 5's fit: cycles per step in rows,
# CHIVI max + barrier, reduce-scatter, barrier, update, end barrier.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06l
VIABEL_AMD_LIB=viabel_amd/libviabel_amd_ts.so timeout -k 10 200 python -u scripts/block_phase_cfg12.py > gpurun_out/r06l/block_ts.log 2>&1 || exit $?
grep -E "==|BLOCKTS|COPYTS" gpurun_out/r06l/block_ts.log | head -60
