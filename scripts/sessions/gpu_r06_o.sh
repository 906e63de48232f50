#!/bin/bash
# Round 6: fused per-step values, second form (no shared counter: the last 32 blocks
# poll their steps' partials until none holds the "not written" pattern) -- the
# switch / headline tests, then the interleaved headline A/B of gpu_r06_n.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TESTS="tests/test_gpu_switches.py tests/test_gpu_headline.py tests/test_gpu_vb.py" LEGS=cfg1 ROUNDS=4 \
  LIBS="notail+VIABEL_AMD_SEP_FUSED_VALUES=0 new+VIABEL_AMD_SEP_FUSED_VALUES=0 new" \
  bash scripts/gpu_ab_legs.sh
