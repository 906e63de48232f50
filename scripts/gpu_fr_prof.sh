# rocprofv3 kernel trace of the config-4 full-rank step (bench_fr.py)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fr -o fr --output-format csv -- python3 scripts/bench_fr.py --steps 10 > gpurun_out/prof_fr.log 2>&1
find gpurun_out/prof_fr -name "*stats*"
