#!/bin/bash
# Round 5, GPU session ad: split-row block kernels with the benchmark modes compiled in
# (HOT) and sep_kernel's advance launches with theirs (ADV), built as
# libviabel_amd_hot.so -- the block / config / headline tests on it, then configs 1, 2, 5
# and the headline against the committed build ("new"), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_hot.so timeout -k 10 700 python -u -m pytest \
  tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_restarts.py tests/test_gpu_notebooks.py \
  tests/test_gpu_ia.py tests/test_gpu_switches.py tests/test_gpu_headline.py tests/test_gpu_wide.py \
  --deselect tests/test_gpu_vb.py::test_gpu_library_was_built_from_these_sources \
  -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_ad.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ad.log
[ $rc -ne 0 ] && exit $rc
LIBS="hot new" LEGS=cfg1,cfg2,cfg5 ROUNDS=4 bash scripts/gpu_ab_legs.sh | tee gpurun_out/ab_ad.log
