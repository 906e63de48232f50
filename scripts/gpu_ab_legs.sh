#!/bin/bash
# Interleaved A/B of library builds on bench.py legs (default cfg1,cfg2,cfg5), fresh
# processes: LIBS="base new" (viabel_amd/libviabel_amd_<name>.so; "new" = the
# default build).  Optional TESTS: a pytest selection run first on the new build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_ab.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -ne 0 ] && exit $rc
fi
# rounds alternate the order (A B, B A, ...): the second process of a back-to-back pair
# measured ~0.15-0.2 us/step slower on the headline with identical libraries
# (profiles/r03/headline_host/ab_position_bias.log)
LIBS_FWD=${LIBS:-base new}
LIBS_REV=$(echo $LIBS_FWD | awk '{for (i = NF; i > 0; i--) printf "%s ", $i}')
for i in $(seq 1 ${ROUNDS:-3}); do
  if [ $((i % 2)) -eq 1 ]; then ORDER=$LIBS_FWD; else ORDER=$LIBS_REV; fi
  for L in $ORDER; do
    # "name+VAR=value": the library plus an environment switch
    name=${L%%+*}; envv=""; [ "$name" != "$L" ] && envv=${L#*+}
    lib=$PWD/viabel_amd/libviabel_amd_$name.so; [ "$name" = new ] && lib=$PWD/viabel_amd/libviabel_amd.so
    env $envv VIABEL_AMD_LIB=$lib timeout -k 10 200 python bench.py --legs ${LEGS:-cfg1,cfg2,cfg5} --no-cpu-baseline \
      --steps 20 --warmup 5 > gpurun_out/ab_legs.json 2> gpurun_out/ab_legs.err || exit $?
    python - "$L" <<'PY'
import json, sys
d = json.loads([l for l in open('gpurun_out/ab_legs.json') if l.startswith('{')][-1])
c = d['configs']
out = {'lib': sys.argv[1], 'headline_us': round(d['ms_per_step'] * 1e3, 3),
       'headline_launch_us': round(d['roofline']['launch_ms_mean'] * 1e3, 2)}
for k in ('cfg1', 'cfg2'):
    if k in c: out[k + '_us'] = round(c[k].get('ms_per_step', float('nan')) * 1e3, 3)
if 'cfg4' in c:
    out['cfg4_ms'] = round(c['cfg4']['ms_per_step'], 4)
if 'cfg5' in c:
    out.update(cfg5_ms=round(c['cfg5']['seconds'] * 1e3, 2), fit_ms=round(c['cfg5']['fit_s'] * 1e3, 2),
               bounds_ms=round(c['cfg5']['bounds_psis_s'] * 1e3, 2))
print(json.dumps(out), flush=True)
PY
  done
done
