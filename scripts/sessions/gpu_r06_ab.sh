#!/bin/bash
# Round 6: separating gpu_r06_aa's two changes -- v1 = the HOT compile-time facts only
# (window pre-sum, CHIVI's pre-drawn log q), new = v1 + the copy wave forming KLVI's step
# size one step ahead -- against the previous commit (base), configs 1, 2 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
LEGS=cfg1,cfg2,cfg5 ROUNDS=2 LIBS="base v1 new" bash scripts/gpu_ab_legs.sh
