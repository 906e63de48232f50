#!/bin/bash
# Interleaved A/B of the config-5 leg (bench.py --legs cfg5, no CPU legs) over
# LIBS (prev = libviabel_amd_prev.so, new = libviabel_amd.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in $(seq 1 ${ROUNDS:-2}); do
  for L in ${LIBS:-prev new}; do
    name=${L%%+*}; envv=""; [ "$name" != "$L" ] && envv=${L#*+}
    lib=$PWD/viabel_amd/libviabel_amd_$name.so; [ "$name" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    out=$(env $envv VIABEL_AMD_LIB=$lib timeout -k 5 200 python bench.py --legs cfg5 --no-cpu-baseline \
          --steps 20 --warmup 5 2>/dev/null | tail -1) || exit $?
    echo "$L $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read())["configs"]["cfg5"]; print("total_ms %.2f fit_ms %.2f bounds_psis_ms %.2f" % (d["seconds"]*1e3, d["fit_s"]*1e3, d["bounds_psis_s"]*1e3))')"
  done
done
