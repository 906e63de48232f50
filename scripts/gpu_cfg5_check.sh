# Config 5: restart parity tests, then the bench's config-5 leg three times
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_restarts.py tests/test_gpu_bounds_psis.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --legs cfg5 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['configs']['cfg5']; print({k: c[k] for k in ('seconds','fit_s','bounds_psis_s')})"
done
