#!/bin/bash
# Round 6: one-pass divergence statistics (Welford / Chan) -- bounds, reference-bounds,
# restart and config-5 parity tests, then the config-5 stage counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06f
timeout -k 10 600 python -u -m pytest tests/test_gpu_bounds_psis.py tests/test_gpu_reference_bounds.py tests/test_gpu_restarts.py tests/test_gpu_notebooks.py "tests/test_gpu_configs.py::test_config5_full_size_records" -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06f/pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_cfg5_pmc.sh > gpurun_out/cfg5_pmc.log 2>&1 || { tail -20 gpurun_out/cfg5_pmc.log; exit 1; }
python3 scripts/summarize_cfg5_pmc.py gpurun_out/cfg5_pmc > gpurun_out/cfg5_pmc/summary.json && python3 -c "
import json; d=json.load(open('gpurun_out/cfg5_pmc/summary.json'))
print(d['stage'])
for k,v in d['kernels'].items(): print('%-60s %8.4f ms valu %.3f' % (k[:60], v['ms'], v['valu_frac'] or 0))"
