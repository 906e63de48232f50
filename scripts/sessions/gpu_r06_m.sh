#!/bin/bash
# Round 6: CHIVI without the block-max barrier (per-wave maxima, the column readers
# rescale the waves' sums) -- block / config / IA / switch / notebook tests, the
# driver's bench command, then the per-wave barrier timestamps (VB_BLOCK_TS build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06m
timeout -k 10 900 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_configs.py tests/test_gpu_ia.py tests/test_gpu_switches.py tests/test_gpu_notebooks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06m/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r06m/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06m/bench.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r06m/bench.log') if l.startswith('{')][-1])
c = d['configs']
print('value', d['value'], 'ms/step', d['ms_per_step'])
for k, v in c.items():
    r = v.get('roofline', {})
    print(k, {kk: v.get(kk) for kk in ('ms_per_step', 'seconds', 'fit_s', 'bounds_psis_s') if kk in v}, 'floor', r.get('floor_us'))
PY
VIABEL_AMD_LIB=viabel_amd/libviabel_amd_ts.so timeout -k 10 200 python -u scripts/block_phase_cfg12.py > gpurun_out/r06m/block_ts.log 2>&1 || exit $?
grep -E "==|BLOCKTS|COPYTS" gpurun_out/r06m/block_ts.log > gpurun_out/r06m/block_ts_lines.log
grep -c BLOCKTS gpurun_out/r06m/block_ts_lines.log
