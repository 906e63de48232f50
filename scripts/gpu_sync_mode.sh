#!/bin/bash
# scripts/sync_mode.py under each HIP scheduling flag, interleaved, fresh processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for f in -1 0 1 2 4; do
    timeout -k 10 120 python scripts/sync_mode.py $f 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
