#!/bin/bash
# Round 5, GPU session t: headline A/B of the sample loop unrolled 2 / 4 times
# (two or four rows' Philox / Box-Muller chains interleaved: the 4-pair wave's step is
# bound by its own dependent chains, not by the SIMD's issue rate) against the
# current build ("new", unroll 1) and the previous commit ("prev").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then ORDER="new u2 u4 prev"; else ORDER="prev u4 u2 new"; fi
  for L in $ORDER; do
    lib=$PWD/viabel_amd/libviabel_amd_$L.so; [ "$L" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    out=$(VIABEL_AMD_LIB=$lib timeout -k 5 120 python bench.py --legs none --no-cpu-baseline \
          --steps 20 --warmup 5 2>/dev/null | tail -1) || exit $?
    echo "lib=$L $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))')"
  done
done | tee gpurun_out/unroll_ab_t.log
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_u2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_vb.py -x -q \
  -k "sep or layouts or philox" --timeout 200 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_t.log
exit $rc
