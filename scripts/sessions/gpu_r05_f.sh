#!/bin/bash
# Round 5, GPU session f: phase stamps of the symmetric-sum PCG launches
# (VB_SS_PROF build), L2 hit / fetch counters of the isolated symmetric-sum and
# plain products, config-5 stage counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_ssprof.so timeout -k 5 120 python scripts/bench_fr.py --steps 12 \
  > gpurun_out/ss_prof.log 2>&1 || exit $?
python scripts/ss_phases.py gpurun_out/ss_prof.log | tee gpurun_out/ss_phases.txt
B=scripts/ubench/symsum_bench
timeout -k 5 60 $B > gpurun_out/symsum_bench.log 2>&1 || exit $?
cat gpurun_out/symsum_bench.log
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/ss_pmc1 -o run --output-format csv -- $B \
  > gpurun_out/ss_pmc1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ss_pmc2 -o run --output-format csv -- $B \
  > gpurun_out/ss_pmc2.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM \
  -d gpurun_out/ss_pmc3 -o run --output-format csv -- $B > gpurun_out/ss_pmc3.log 2>&1 || exit $?
bash scripts/gpu_cfg5_pmc.sh > gpurun_out/cfg5_pmc.log 2>&1 || exit $?
tail -3 gpurun_out/cfg5_pmc.log
