#!/bin/bash
# Round-4: config-5 fit split (pre-draw vs block kernel, rocprofv3 kernel stats) and
# block-kernel barrier timestamps of configs 1, 2 and 5's fit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_cfg5fit
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg5fit -o fit --output-format csv -- \
  python3 scripts/cfg5_fit_split.py > gpurun_out/prof_cfg5fit.log 2>&1 || { tail -5 gpurun_out/prof_cfg5fit.log; exit 1; }
tail -2 gpurun_out/prof_cfg5fit.log
f=$(find gpurun_out/prof_cfg5fit -name "*kernel_stats.csv" | head -1)
head -8 "$f" | cut -c1-200
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_ts.so timeout -k 10 120 python -u scripts/block_phase_cfg12.py \
  > gpurun_out/block_ts3.log 2>&1 || exit 1
grep -E "==|BLOCKTS" gpurun_out/block_ts3.log | grep -v "steps=512" | head -20
