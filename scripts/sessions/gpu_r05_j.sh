#!/bin/bash
# Round 5, GPU session j: headline (20-step launch) under the column-pair layouts
# of VB_SEP_MODE (default "q" = one 4-pair wave + 1-pair waves per SIMD; "mix" =
# two 2-pair waves + 1-pair waves; all 2-pair; all 1-pair), alternating order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then ORDER="q mix 2 1"; else ORDER="1 2 mix q"; fi
  for M in $ORDER; do
    if [ "$M" = q ]; then E="VB_SEP_MODE_UNSET=1"; else E="VB_SEP_MODE=$M"; fi
    out=$(env $E timeout -k 5 120 python bench.py --legs none --no-cpu-baseline --steps 20 --warmup 5 \
          2>/dev/null | tail -1) || exit $?
    echo "mode=$M $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))')"
  done
done | tee gpurun_out/sep_mode_ab.log
