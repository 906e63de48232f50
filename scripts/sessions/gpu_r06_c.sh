#!/bin/bash
# Round 6: polar t log-weight draws, sharded IA / R-hat, teardown: their tests, the
# restart / config-5 / PSIS suites, then the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06c
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_polar.py tests/test_gpu_ia_dist.py tests/test_gpu_teardown.py tests/test_gpu_restarts.py tests/test_gpu_bounds_psis.py tests/test_gpu_ia.py "tests/test_gpu_configs.py::test_config5_full_size_records" -x -v --timeout 300 --timeout-method thread > gpurun_out/r06c/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r06c/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06c/bench.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r06c/bench.log') if l.startswith('{')][-1])
c = d['configs']
print('value', d['value'], 'ms/step', d['ms_per_step'])
for k, v in c.items():
    print(k, {kk: v.get(kk) for kk in ('ms_per_step', 'us_per_step', 'total_ms', 'fit_ms', 'bounds_psis_ms', 'value') if kk in v})
PY
# register-direct small-tile GEMM probe (built in-tree: scripts/ubench/gemm_rd)
timeout -k 10 120 ./scripts/ubench/gemm_rd > gpurun_out/r06c/gemm_rd.log 2>&1; cat gpurun_out/r06c/gemm_rd.log
