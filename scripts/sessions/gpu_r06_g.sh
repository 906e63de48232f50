#!/bin/bash
# Round 6: Bailey trigonometric t log-weight draws + two-pass divergence form -- their
# tests, the restart / bounds / config-5 parity tests, the switch test, then the
# config-5 stage counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06g
timeout -k 10 700 python -u -m pytest tests/test_gpu_bailey.py tests/test_gpu_restarts.py tests/test_gpu_bounds_psis.py tests/test_gpu_reference_bounds.py "tests/test_gpu_switches.py::test_div_two_pass_switch" "tests/test_gpu_configs.py::test_config5_full_size_records" tests/test_gpu_vb.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06g/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06g/pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_cfg5_pmc.sh > gpurun_out/cfg5_pmc.log 2>&1 || { tail -20 gpurun_out/cfg5_pmc.log; exit 1; }
python3 scripts/summarize_cfg5_pmc.py gpurun_out/cfg5_pmc > gpurun_out/cfg5_pmc/summary.json && python3 -c "
import json; d=json.load(open('gpurun_out/cfg5_pmc/summary.json'))
print(d['stage'])
for k,v in list(d['kernels'].items())[:6]: print('%-60s %8.4f ms valu %.3f instr %.3g' % (k[:60], v['ms'], v['valu_frac'] or 0, v['valu_instr']))"
