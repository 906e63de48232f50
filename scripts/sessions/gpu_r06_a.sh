#!/bin/bash
# Round 6, first call: the driver's bench command on the round-5 tree (baseline of
# this box), then scripts/teardown_child.py (>= 8-problem run, exits without
# release_all) plain and under rocprofv3 --kernel-trace, to reproduce the round-5
# teardown crash before the library fix.  Each GPU step has its own limit; the
# first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06a/bench.log 2>&1 || exit $?
tail -c 400 gpurun_out/r06a/bench.log
timeout -k 10 300 python -u scripts/teardown_child.py > gpurun_out/r06a/child_plain.log 2>&1
echo "plain rc=$?"; tail -2 gpurun_out/r06a/child_plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06a/prof -o child -- python3 -u scripts/teardown_child.py > gpurun_out/r06a/child_prof.log 2>&1
echo "rocprofv3 rc=$?"; tail -4 gpurun_out/r06a/child_prof.log
