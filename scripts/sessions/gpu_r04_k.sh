#!/bin/bash
# Round-4 overlapped pre-draw (CU-masked streams): bitwise test against the serial
# order, the config / restart tests, then an interleaved A/B of configs 2 and 5
# (VIABEL_AMD_PREDRAW_OVERLAP=0 vs on).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_vb.py -k "overlap or predraw" tests/test_gpu_restarts.py tests/test_gpu_configs.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_k.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg2,cfg5 LIBS="new+VIABEL_AMD_PREDRAW_OVERLAP=0 new" ROUNDS=4 bash scripts/gpu_ab_legs.sh > gpurun_out/predraw_overlap_ab.log 2>&1 || { cat gpurun_out/predraw_overlap_ab.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/predraw_overlap_ab.log
