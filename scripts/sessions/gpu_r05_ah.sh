#!/bin/bash
# Round 5, GPU session ah: smoke() and the driver's bench command on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/rec2
export TMPDIR=/tmp
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rec2/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/rec2/smoke.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rec2/bench.log 2>&1 || exit $?
tail -c 200 gpurun_out/rec2/bench.log
