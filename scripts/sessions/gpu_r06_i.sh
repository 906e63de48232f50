#!/bin/bash
# Round 6: Bailey transform trimmed (three-address constants, integer cosine table
# point, no expm1 clamp) -- block / config / Bailey / restart / wide tests, then the
# config-5 stage counter passes and the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06i
timeout -k 10 900 python -u -m pytest tests/test_gpu_bailey.py tests/test_gpu_restarts.py tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06i/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06i/pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_cfg5_pmc.sh > gpurun_out/cfg5_pmc.log 2>&1 || { tail -20 gpurun_out/cfg5_pmc.log; exit 1; }
python3 scripts/summarize_cfg5_pmc.py gpurun_out/cfg5_pmc > gpurun_out/cfg5_pmc/summary.json && python3 -c "
import json; d=json.load(open('gpurun_out/cfg5_pmc/summary.json'))
print(d['stage'])
for k,v in list(d['kernels'].items())[:3]: print('%-60s %8.4f ms valu %.3f instr %.3g' % (k[:60], v['ms'], v['valu_frac'] or 0, v['valu_instr']))"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06i/bench.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r06i/bench.log') if l.startswith('{')][-1])
c = d['configs']
print('value', d['value'], 'ms/step', d['ms_per_step'])
for k, v in c.items():
    print(k, {kk: v.get(kk) for kk in ('ms_per_step', 'seconds', 'fit_s', 'bounds_psis_s') if kk in v})
PY
