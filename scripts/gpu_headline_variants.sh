#!/bin/bash
# Headline us/step of bench.py under different flags (fresh processes, rotating order):
# does anything outside the timed region change it?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 "$@" > gpurun_out/hv.json 2> gpurun_out/hv.err || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/hv.json') if l.startswith('{')][-1]); print(json.dumps({'flags': '$*', 'headline_us': round(d['ms_per_step']*1e3, 3), 'launch_us': round(d['roofline']['launch_ms_mean']*1e3, 2)}))"
}
for i in 1 2 3; do
  run --legs none --no-cpu-baseline
  run --legs none
  run --legs cfg1 --no-cpu-baseline
done
