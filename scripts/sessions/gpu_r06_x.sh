#!/bin/bash
# Round 6: interleaved A/B of the stream-K wait's NaN poisoning (new) against the
# previous commit's vb_gemm.hpp (prev) on configs 4 and 5 (box-to-box spread check).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
LEGS=cfg4,cfg5 ROUNDS=3 LIBS="prev new" bash scripts/gpu_ab_legs.sh
