#!/bin/bash
# Round 5, GPU session d: all gpu tests on the current tree; config-4 A/B of the PCG
# loops and its step timeline; headline A/B of the lambda / window prefetch (new
# vs nopre); configs 1 / 2 / 5 A/B of the CHIVI provisional shift (new vs chivi0 =
# round 4's block-max barrier); the driver's bench command.  Stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for E in "VIABEL_AMD_FR_PCG_SS=0" "VIABEL_AMD_FR_PCG_SS=1"; do
    echo -n "[$E] "; env $E timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
OUT=gpurun_out/prof_fr bash scripts/gpu_cfg4_timeline.sh || exit $?
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 1 ]; then ORDER="new nopre"; else ORDER="nopre new"; fi
  for L in $ORDER; do
    lib=$PWD/viabel_amd/libviabel_amd_$L.so; [ "$L" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    out=$(VIABEL_AMD_LIB=$lib timeout -k 5 120 python bench.py --legs none --no-cpu-baseline \
          --steps 20 --warmup 5 2>/dev/null | tail -1) || exit $?
    echo "lib=$L $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))')"
  done
done | tee gpurun_out/headline_ab_d.log
LIBS="new chivi0" LEGS=cfg1,cfg2,cfg5 ROUNDS=3 bash scripts/gpu_ab_legs.sh | tee gpurun_out/legs_ab_d.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench.log
