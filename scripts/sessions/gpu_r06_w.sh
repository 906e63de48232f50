#!/bin/bash
# Round 6: the floor skeleton's KLVI pre-sum placement as block_kernel's, and the stream-K
# wait's NaN poisoning on a (never expected) timeout -- config / full-rank / switch
# tests, then the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06w
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_fullrank.py tests/test_gpu_switches.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06w/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06w/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06w/bench.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r06w/bench.log') if l.startswith('{')][-1])
c = d['configs']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'launch', d['roofline']['launch_ms_mean'])
for k, v in c.items():
    r = v.get('roofline', {})
    print(k, {kk: v.get(kk) for kk in ('ms_per_step', 'seconds', 'fit_s', 'bounds_psis_s') if kk in v}, 'floor', r.get('floor_us'))
PY
