#!/bin/bash
# Round 5, GPU session c: DMA-interleave microbenchmarks; full-rank / headline tests on the new PCG epilogue; config-4
# A/B (PCG_SS 0 / 1) + step timeline; interleaved headline A/B of library builds
# (new = hipExtLaunchKernel events, evrec = event records, prio / prio1 = s_setprio
# 2 / 1 on the 4-pair waves), order alternating each round.  Stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench/hbm_probe2 > gpurun_out/hbm_probe2.log 2>&1 || exit $?
cat gpurun_out/hbm_probe2.log
# LDS-DMA issue interleaved with the MFMA steps vs issued after the barrier
for b in gemm_chain_base gemm_chain_il; do
  echo "[$b]"; timeout -k 10 60 ./scripts/ubench/$b 512 0 || exit $?
done
for b in symsum_bench_gs2 symsum_bench_il; do
  echo "[$b]"; timeout -k 10 60 ./scripts/ubench/$b 512 128 || exit $?
done
for b in gemm_chain_il gemm_chain_base; do
  echo "[$b]"; timeout -k 10 60 ./scripts/ubench/$b 512 0 || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_headline.py tests/test_gpu_configs.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_c.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for E in "VIABEL_AMD_FR_PCG_SS=0" "VIABEL_AMD_FR_PCG_SS=1"; do
    echo -n "[$E] "; env $E timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
OUT=gpurun_out/prof_fr bash scripts/gpu_cfg4_timeline.sh || exit $?
LIBS_FWD="new evrec prio prio1"
LIBS_REV="prio1 prio evrec new"
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then ORDER=$LIBS_FWD; else ORDER=$LIBS_REV; fi
  for L in $ORDER; do
    lib=$PWD/viabel_amd/libviabel_amd_$L.so; [ "$L" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    out=$(VIABEL_AMD_LIB=$lib timeout -k 5 120 python bench.py --legs none --no-cpu-baseline \
          --steps 20 --warmup 5 2>/dev/null | tail -1) || exit $?
    echo "lib=$L $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))')"
  done
done | tee gpurun_out/headline_ab_c.log
# CHIVI with the provisional shift (libviabel_amd_chivi.so = the current sources):
# block-kernel CHIVI tests, then an interleaved A/B of configs 1 / 2 / 5
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_chivi.so timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_notebooks.py tests/test_gpu_ia.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_chivi.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_chivi.log; [ $rc -ne 0 ] && exit $rc
LIBS="new chivi" LEGS=cfg1,cfg2,cfg5 ROUNDS=3 bash scripts/gpu_ab_legs.sh
