#!/bin/bash
# Round 5, GPU session q: where the HIP runtime puts kernel arguments -- config 4 and
# the headline with HIP_FORCE_DEV_KERNARG unset / 1 / 0, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for E in "KA_UNSET=1" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0"; do
    echo -n "[$E] cfg4 "; env $E timeout -k 5 120 python scripts/bench_fr.py --steps 40 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    out=$(env $E timeout -k 5 120 python bench.py --legs none --no-cpu-baseline --steps 20 --warmup 5 2>/dev/null | tail -1) || exit $?
    echo "[$E] headline $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f launch_us %.2f" % (d["ms_per_step"]*1e3, r["launch_ms_mean"]*1e3))')"
  done
done | tee gpurun_out/kernarg_ab.log
