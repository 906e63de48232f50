#!/bin/bash
# Round 5, GPU session o: column-pair tests after the layout switch's removal
# (every branch of the grid split against the oracle), the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_vb.py tests/test_gpu_headline.py -x -q \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_o.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_o.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 5 120 python bench.py --legs none --no-cpu-baseline --steps 20 --warmup 5 2>/dev/null | tail -1 | \
    python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))' || exit 1
done
