#!/bin/bash
# Round 5, GPU session a: the symmetric-sum product microbenchmark (correctness +
# time against the plain product), the full-rank tests with the new PCG loop,
# an interleaved config-4 A/B (VIABEL_AMD_FR_PCG_SS=0 vs default), all gpu tests,
# the driver's bench command, per-wave timestamps of the headline launch, and a
# config-4 step timeline.  Each GPU step has its own limit; stop at the first
# failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench/symsum_bench 512 > gpurun_out/symsum_bench.log 2>&1 || exit $?
cat gpurun_out/symsum_bench.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_headline.py -x -q \
  --timeout 300 --timeout-method thread -k "fullrank or config4 or full_rank" > gpurun_out/pytest_fr.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fr.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for E in "VIABEL_AMD_FR_PCG_SS=0" "VIABEL_AMD_FR_PCG_SS=1"; do
    echo -n "[$E] "; env $E timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
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
OUT=gpurun_out/prof_fr bash scripts/gpu_cfg4_timeline.sh
