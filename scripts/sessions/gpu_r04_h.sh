#!/bin/bash
# Round-4 split rows (two lanes per sample in the block kernel's copy-wave layout):
# the block-kernel parity tests, then configs 1 / 2 / 5 with and without the split
# (VIABEL_AMD_BLOCK_SPLIT=0), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_notebooks.py tests/test_gpu_restarts.py tests/test_gpu_ia.py tests/test_gpu_callback.py tests/test_gpu_wide.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_h.log; [ $rc -ne 0 ] && exit $rc
LIBS="prev new" ROUNDS=4 bash scripts/gpu_ab_legs.sh > gpurun_out/block_split_ab.log 2>&1 || { cat gpurun_out/block_split_ab.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/block_split_ab.log
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_ts.so timeout -k 10 120 python -u scripts/block_phase_cfg12.py \
  > gpurun_out/block_ts_split.log 2>&1 || exit 1
grep -E "==|BLOCKTS" gpurun_out/block_ts_split.log | head -12
