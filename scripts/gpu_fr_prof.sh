set -e
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 300 python scripts/bench_fr.py --steps 20 --cpu > gpurun_out/bench_fr.json 2> gpurun_out/bench_fr.err
timeout -k 10 300 python scripts/bench_fr.py --steps 20 --objective klvi >> gpurun_out/bench_fr.json 2>> gpurun_out/bench_fr.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fr -o fr -- python3 scripts/bench_fr.py --steps 10 > gpurun_out/prof_fr.log 2>&1
find gpurun_out/prof_fr -name "*kernel_stats.csv" | head
