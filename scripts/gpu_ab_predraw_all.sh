#!/bin/bash
# Interleaved A/B: config 1 (Gaussian family) with in-kernel draw waves (default)
# vs pre-drawn noise through the copy-wave path (VIABEL_AMD_PREDRAW=all).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-3}); do
  for pd in t all; do
    VIABEL_AMD_PREDRAW=$pd timeout -k 10 200 python bench.py --legs cfg1 --no-cpu-baseline \
      --steps 20 --warmup 5 > gpurun_out/ab_pd.json 2> gpurun_out/ab_pd.err || exit $?
    python - "$pd" <<'PY'
import json, sys
d = json.loads([l for l in open('gpurun_out/ab_pd.json') if l.startswith('{')][-1])
c = d['configs']['cfg1']
print(json.dumps({'predraw': sys.argv[1], 'cfg1_us': round(c['ms_per_step'] * 1e3, 3),
                  'floor_us': (c.get('roofline') or {}).get('floor_us')}), flush=True)
PY
  done
done
