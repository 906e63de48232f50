#!/bin/bash
# Round 5, GPU session r: column-pair / block tests; headline and legs A/B of the
# straight-line LDS table fill + kernarg warm-up in sep_kernel ("new") against the
# previous commit ("prev").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_headline.py tests/test_gpu_configs.py -x -q \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_r.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 1 ]; then ORDER="new prev"; else ORDER="prev new"; fi
  for L in $ORDER; do
    lib=$PWD/viabel_amd/libviabel_amd_$L.so; [ "$L" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    out=$(VIABEL_AMD_LIB=$lib timeout -k 5 120 python bench.py --legs none --no-cpu-baseline \
          --steps 20 --warmup 5 2>/dev/null | tail -1) || exit $?
    echo "lib=$L $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))')"
  done
done | tee gpurun_out/headline_ab_r.log
LIBS="new prev" LEGS=cfg1,cfg2 ROUNDS=2 bash scripts/gpu_ab_legs.sh | tee gpurun_out/legs_ab_r.log
