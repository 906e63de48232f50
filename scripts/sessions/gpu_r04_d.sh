#!/bin/bash
# Round-4 headline: per-step values inside sep_kernel for short launches.  Headline
# and sep-path tests, then an interleaved A/B of the driver's headline command
# (bench.py --legs none) with VIABEL_AMD_SEP_FUSE_VALUES=0 vs default, alternating
# the order each round.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_vb.py tests/test_gpu_wide.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_d.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_d.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 1 ]; then order="0 1"; else order="1 0"; fi
  for f in $order; do
    out=$(VIABEL_AMD_SEP_FUSE_VALUES=$f timeout -k 5 120 python bench.py --legs none --no-cpu-baseline \
          --steps 20 --warmup 5 2>/dev/null | tail -1) || exit $?
    echo "fuse=$f $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))')"
  done
done | tee gpurun_out/headline_fuse_ab.log
