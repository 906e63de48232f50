#!/bin/bash
# Round 5, GPU session b: symmetric-sum product variants (stage depth 64 / 128 x
# 2 / 3 stages) against the plain product; config-4 A/B of the PCG loops and
# its step timeline; then all gpu tests, the driver's bench command and the
# headline's per-wave timestamps.  Stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for gs in 2 3; do for kt in 64 128; do
  timeout -k 10 60 ./scripts/ubench/symsum_bench_gs$gs 512 $kt >> gpurun_out/symsum_bench.log 2>&1 || exit $?
done; done
cat gpurun_out/symsum_bench.log
for i in 1 2 3; do
  for E in "VIABEL_AMD_FR_PCG_SS=0" "VIABEL_AMD_FR_PCG_SS=1"; do
    echo -n "[$E] "; env $E timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
OUT=gpurun_out/prof_fr bash scripts/gpu_cfg4_timeline.sh || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/bench.log
for s in 20 256; do
  VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_septs.so timeout -k 10 120 python scripts/sep_steps_ts.py $s \
    > gpurun_out/septs_$s.log 2>&1 || exit $?
done
cat gpurun_out/septs_20.log
