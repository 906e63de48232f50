#!/bin/bash
# Round 5, GPU session i: config-4 A/B of the symmetric-sum block order (XCD-grouped
# = default vs geo order = noxcd build), alternating; plain GEMM chain with and
# without the XCD rectangle order; per-wave timeline of a 20-step headline launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then ORDER="new noxcd"; else ORDER="noxcd new"; fi
  for L in $ORDER; do
    lib=$PWD/viabel_amd/libviabel_amd_$L.so; [ "$L" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    echo -n "[$L] "; VIABEL_AMD_LIB=$lib timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee gpurun_out/cfg4_xcd_ab.log
for i in 1 2; do
  for B in gemm_chain gemm_chain_xcd; do
    echo -n "[$B] "; timeout -k 5 60 scripts/ubench/$B 512 0 2>&1 | tail -1 || exit 1
  done
done | tee gpurun_out/gemm_xcd_ab.log
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_sepprof.so timeout -k 5 120 python scripts/sep_timeline.py 20 \
  > gpurun_out/sep_prof.log 2>&1 || exit $?
python scripts/sep_timeline.py --parse gpurun_out/sep_prof.log | tee gpurun_out/sep_timeline.txt
