#!/bin/bash
# Round 6: general stream-K (any number of parts per tile) for the Newton-Schulz T and
# Y|Z products and the N-row x / target products -- full-rank / config-4 / switch tests,
# interleaved config-4 A/B against the two-part Y|Z-only form (libviabel_amd_sk2.so),
# then the config-4 step timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06s
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_configs.py tests/test_gpu_headline.py "tests/test_gpu_switches.py::test_gemm_sk_off_matches_default" "tests/test_gpu_switches.py::test_full_rank_switch_off_matches_default" -x -q --timeout 300 --timeout-method thread > gpurun_out/r06s/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06s/pytest.log; [ $rc -ne 0 ] && exit $rc
LEGS=cfg4 ROUNDS=3 LIBS="sk2 new" bash scripts/gpu_ab_legs.sh || exit $?
OUT=gpurun_out/r06s/prof_fr bash scripts/gpu_cfg4_timeline.sh
