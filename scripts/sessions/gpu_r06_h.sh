#!/bin/bash
# Round 6: Bailey draws with the cosine-only table -- the Bailey / restart tests, then
# the driver's bench command (config-5 bounds stage in the line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06h
timeout -k 10 300 python -u -m pytest tests/test_gpu_bailey.py tests/test_gpu_restarts.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06h/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06h/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06h/bench.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r06h/bench.log') if l.startswith('{')][-1])
c = d['configs']
print('value', d['value'], 'ms/step', d['ms_per_step'])
for k, v in c.items():
    print(k, {kk: v.get(kk) for kk in ('ms_per_step', 'seconds', 'fit_s', 'bounds_psis_s') if kk in v})
PY
