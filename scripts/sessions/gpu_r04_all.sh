#!/bin/bash
# Round-4 combined GPU pass: the full -m gpu suite, smoke(), then the A/Bs of this
# round's changes (scripts/sessions/gpu_r04_b.sh minus its tests, scripts/sessions/gpu_r04_c.sh, scripts/sessions/gpu_r04_d.sh
# A/B parts).  Each GPU step has its own limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "full suite rc=$rc"; tail -3 gpurun_out/pytest_all.log; [ $rc -ne 0 ] && exit $rc
VIABEL_AMD_FR_WEIGHTS_FUSE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_configs.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_wfuse.log 2>&1
rc=$?; echo "weights-fused fr tests rc=$rc"; tail -2 gpurun_out/pytest_wfuse.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
for i in 1 2; do
  echo old; timeout -k 5 60 ./scripts/ubench/gemm_chain_old 512 || exit $?
  echo new; timeout -k 5 60 ./scripts/ubench/gemm_chain 512 || exit $?
done > gpurun_out/gemm_chain_ab.log 2>&1
cat gpurun_out/gemm_chain_ab.log
timeout -k 5 60 ./scripts/ubench/gemm_phase 0 0 > gpurun_out/gemm_phase_b.log 2>&1 || exit $?
timeout -k 5 60 ./scripts/ubench/gemm_phase 1 1 >> gpurun_out/gemm_phase_b.log 2>&1 || exit $?
grep -E "span|loop end|acc summed|epi operands|tile stored|epilogue end" gpurun_out/gemm_phase_b.log
LIBS="base new" ROUNDS=3 bash scripts/gpu_ab_fr2.sh > gpurun_out/fr_ab_epi.log 2>&1 || exit $?
cat gpurun_out/fr_ab_epi.log
ENVA="" ENVB="VIABEL_AMD_FR_WEIGHTS_FUSE=1" ROUNDS=3 bash scripts/gpu_ab_env.sh > gpurun_out/fr_ab_w.log 2>&1 || exit $?
cat gpurun_out/fr_ab_w.log
LIBS="pairloops new" ROUNDS=3 bash scripts/gpu_ab_cfg5.sh 2>&1 | tee gpurun_out/cfg5_ab.log
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 1 ]; then order="0 1"; else order="1 0"; fi
  for f in $order; do
    out=$(VIABEL_AMD_SEP_FUSE_VALUES=$f timeout -k 5 120 python bench.py --legs none --no-cpu-baseline \
          --steps 20 --warmup 5 2>/dev/null | tail -1) || exit $?
    echo "fuse=$f $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("us_per_step %.3f value %.4g launch_us %.2f" % (d["ms_per_step"]*1e3, d["value"], r["launch_ms_mean"]*1e3))')"
  done
done | tee gpurun_out/headline_fuse_ab.log
