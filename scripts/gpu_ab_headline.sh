#!/bin/bash
# Interleaved A/B of the driver's headline command (bench.py --steps 20
# --warmup 5, headline only, no CPU legs), one fresh process per run:
# LIBS="prev new" bash scripts/gpu_ab_headline.sh   (new = libviabel_amd.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in $(seq 1 ${ROUNDS:-4}); do
  for L in ${LIBS:-prev new}; do
    # L = lib name [+ENV=VALUE]: new = libviabel_amd.so
    name=${L%%+*}; envv=""; [ "$name" != "$L" ] && envv=${L#*+}
    lib=$PWD/viabel_amd/libviabel_amd_$name.so; [ "$name" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    out=$(env $envv VIABEL_AMD_LIB=$lib timeout -k 5 120 python bench.py --legs none --no-cpu-baseline \
          --steps ${STEPS:-20} --warmup ${WARMUP:-5} 2>/dev/null | tail -1) || exit $?
    echo "$L $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("us_per_step %.3f launch_us %.2f value %.3e" % (d["ms_per_step"]*1e3, d["roofline"]["launch_ms_mean"]*1e3, d["value"]))')"
  done
done
