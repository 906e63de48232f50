#!/bin/bash
# Round 6: fused per-step values of the column-pair kernel (sep_values_tail) -- the
# switch / config tests, then an interleaved headline A/B of three legs: the build
# without the tail code (unfused), the default build unfused (VIABEL_AMD_SEP_FUSED_VALUES=0),
# the default build fused; config 2 after reverting the per-wave CHIVI max.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TESTS="tests/test_gpu_switches.py tests/test_gpu_configs.py" LEGS=cfg2 ROUNDS=4 \
  LIBS="notail+VIABEL_AMD_SEP_FUSED_VALUES=0 new+VIABEL_AMD_SEP_FUSED_VALUES=0 new" \
  bash scripts/gpu_ab_legs.sh
