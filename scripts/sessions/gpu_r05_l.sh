#!/bin/bash
# Round 5, GPU session l: headline counter passes on the current sep_kernel --
# FETCH_SIZE / WRITE_SIZE / SQ passes at N = 128 and 256 over 5-, 256- and 20-step
# launches (scripts/profile_r02.sh PASSES=pmc -> per-launch traffic / VALU models)
# and the VALU-busy pass over the driver's headline command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof2
PASSES=pmc bash scripts/profile_r02.sh > gpurun_out/prof2_pmc.log 2>&1 || exit $?
tail -3 gpurun_out/prof2_pmc.log
bash scripts/gpu_valu_busy.sh > gpurun_out/valu_busy.log 2>&1 || exit $?
tail -5 gpurun_out/valu_busy.log
