#!/bin/bash
# Round-6 record of the tree after the closing host-path changes (device block cache,
# lazy family RandomState, restart table in one op, warm-ups at the timed shapes):
# the whole -m gpu suite, smoke(), the driver's bench command, and the rocprofv3
# kernel trace + stats of the same command.  Outputs under gpurun_out/rec_close/.
# Each GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rec_close
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/rec_close/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/rec_close/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rec_close/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/rec_close/smoke.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rec_close/bench.log 2>&1 || exit $?
tail -c 300 gpurun_out/rec_close/bench.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/rec_close/trace -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rec_close/trace.log 2>&1 || exit $?
find gpurun_out/rec_close/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/rec_close/driver_cmd_kernel_stats.csv \;
ls gpurun_out/rec_close
