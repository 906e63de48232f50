#!/bin/bash
# Interleaved A/B of the block kernel's device-noise copy wave (VIABEL_AMD_BLOCK_PF):
# bench.py's config-2 and config-5 legs in fresh processes, then the block-path
# GPU tests with the default.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_vb.py tests/test_gpu_restarts.py tests/test_gpu_configs.py} \
  -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_pf.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_pf.log; [ $rc -ne 0 ] && exit $rc
for i in $(seq 1 ${ROUNDS:-3}); do
  for pf in 0 1; do
    VIABEL_AMD_BLOCK_PF=$pf timeout -k 10 200 python bench.py --legs ${LEGS:-cfg1,cfg2,cfg5} --no-cpu-baseline \
      --steps 20 --warmup 5 > gpurun_out/ab_pf_$pf.json 2> gpurun_out/ab_pf_$pf.err || exit $?
    python - "$pf" <<'PY'
import json, sys
d = json.loads([l for l in open('gpurun_out/ab_pf_%s.json' % sys.argv[1]) if l.startswith('{')][-1])
c = d['configs']
out = {'pf': sys.argv[1]}
for k in ('cfg1', 'cfg2'):
    if k in c: out[k + '_us'] = round(c[k].get('ms_per_step', float('nan')) * 1e3, 3)
if 'cfg5' in c:
    out.update(cfg5_ms=round(c['cfg5']['seconds'] * 1e3, 2), fit_ms=round(c['cfg5']['fit_s'] * 1e3, 2),
               bounds_ms=round(c['cfg5']['bounds_psis_s'] * 1e3, 2))
print(json.dumps(out), flush=True)
PY
  done
done
