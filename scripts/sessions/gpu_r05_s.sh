#!/bin/bash
# Round 5, GPU session s: tests of the column-pair, block and full-rank paths; A/B of
# "new" (straight-line LDS table fill, kernarg warm-up and isotropic-Gaussian moment
# sums in sep_kernel; the PCG
# kernel's first-stage arguments preloaded into SGPRs) against the previous commit
# ("prev") on the headline, config 4 and configs 1 / 2; phase stamps of the PCG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_headline.py tests/test_gpu_configs.py \
  tests/test_gpu_fullrank.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_s.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 1 ]; then ORDER="new prev"; else ORDER="prev new"; fi
  for L in $ORDER; do
    lib=$PWD/viabel_amd/libviabel_amd_$L.so; [ "$L" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    out=$(VIABEL_AMD_LIB=$lib timeout -k 5 120 python bench.py --legs none --no-cpu-baseline \
          --steps 20 --warmup 5 2>/dev/null | tail -1) || exit $?
    echo "lib=$L $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))')"
    echo -n "lib=$L cfg4 "; VIABEL_AMD_LIB=$lib timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee gpurun_out/ab_s.log
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_ssprof.so timeout -k 5 120 python scripts/bench_fr.py --steps 12 \
  > gpurun_out/ss_prof_s.log 2>&1 || exit $?
python scripts/ss_phases.py gpurun_out/ss_prof_s.log | tail -8
LIBS="new prev" LEGS=cfg1,cfg2 ROUNDS=2 bash scripts/gpu_ab_legs.sh | tee gpurun_out/legs_ab_s.log
