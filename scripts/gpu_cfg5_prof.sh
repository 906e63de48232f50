# rocprofv3 kernel trace + stats of the config-5 leg alone (gpurun_out/prof_cfg5/)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg5 -o c5 --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --legs cfg5 > gpurun_out/prof_cfg5.log 2>&1
find gpurun_out/prof_cfg5 -name "*stats*"
