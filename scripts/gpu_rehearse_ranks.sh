#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: N ranks share the GPU over the
# gloo backend (RCCL refuses two ranks on one GPU), each rank runs the headline restart
# and its share of the config-5 restarts; prints each run's summary.  Correctness only:
# the ranks contend for one GPU, so the numbers are not a scaling measurement.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# (bench.py picks gloo itself when local ranks outnumber the GPUs)
for n in ${RANKS:-2 4}; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 \
    > gpurun_out/rehearse_$n.log 2> gpurun_out/rehearse_$n.err || { tail -20 gpurun_out/rehearse_$n.err; exit 1; }
  python - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads([l for l in open('gpurun_out/rehearse_%s.log' % n) if l.startswith('{')][-1])
c = d['configs'].get('cfg5', {})
print(json.dumps({'ranks': n, 'n_gpus': d['n_gpus'], 'value': d['value'], 'ms_per_step': d['ms_per_step'],
                  'restart_summaries': d['restart_summaries'],
                  'cfg5': {k: c.get(k) for k in ('seconds', 'fit_s', 'bounds_psis_s', 'khat_range',
                                                 'finite_khat', 'error')}}), flush=True)
PY
done
