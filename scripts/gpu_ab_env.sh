#!/bin/bash
# Interleaved A/B of an environment switch on bench_fr.py (config 4):
# ENVA="VIABEL_AMD_FR_FUSE=0" ENVB="" bash scripts/gpu_ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in $(seq 1 ${ROUNDS:-3}); do
  for E in "${ENVA:-}" "${ENVB:-}"; do
    echo -n "env=[$E] "; env $E timeout -k 5 120 python scripts/bench_fr.py --steps ${STEPS:-40} 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
