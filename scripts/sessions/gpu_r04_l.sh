#!/bin/bash
# Round-4 pre-draw overlap: CU-mask layouts on configs 1, 2 and 5 (interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LEGS=cfg1,cfg2,cfg5 LIBS="new+VIABEL_AMD_PREDRAW_OVERLAP=0 new" ROUNDS=3 \
  bash scripts/gpu_ab_legs.sh > gpurun_out/predraw_overlap_ab2.log 2>&1 || { cat gpurun_out/predraw_overlap_ab2.log; tail gpurun_out/ab_legs.err; exit 1; }
cat gpurun_out/predraw_overlap_ab2.log
