#!/bin/bash
# Round 5, GPU session n: full-rank tests; config-4 A/B of the PCG kernel prologue
# (first stage issued before the epilogue's loads, one kernarg batch: "new") against
# the last committed PCG ("prev"); phase stamps of the new prologue.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_n.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_n.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then ORDER="new prev"; else ORDER="prev new"; fi
  for L in $ORDER; do
    lib=$PWD/viabel_amd/libviabel_amd_$L.so; [ "$L" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    echo -n "[$L] "; VIABEL_AMD_LIB=$lib timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee gpurun_out/cfg4_prologue_ab.log
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_ssprof.so timeout -k 5 120 python scripts/bench_fr.py --steps 12 \
  > gpurun_out/ss_prof_n.log 2>&1 || exit $?
python scripts/ss_phases.py gpurun_out/ss_prof_n.log | tail -8
