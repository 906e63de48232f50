#!/bin/bash
# Round 5, GPU session m: headline layout A/B -- default "q" (pairs past 1 024 in
# 4-pair waves, rounded: 992 waves) vs "Q" (4 096 pairs in 4-pair waves: one per SIMD).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 1 ]; then ORDER="q Q"; else ORDER="Q q"; fi
  for M in $ORDER; do
    if [ "$M" = q ]; then E="VB_SEP_MODE_UNSET=1"; else E="VB_SEP_MODE=$M"; fi
    out=$(env $E timeout -k 5 120 python bench.py --legs none --no-cpu-baseline --steps 20 --warmup 5 \
          2>/dev/null | tail -1) || exit $?
    echo "mode=$M $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))')"
  done
done | tee gpurun_out/sep_mode_ab_m.log
