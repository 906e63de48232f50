# One SQ PMC pass over the cold-operand GEMM chain (single 512^3 products)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
./scripts/ubench/gemm_chain 512 0
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_gemm -o g --output-format csv -- ./scripts/ubench/gemm_chain 512 0 > gpurun_out/pmc_gemm.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM -d gpurun_out/pmc_gemm2 -o g --output-format csv -- ./scripts/ubench/gemm_chain 512 0 > gpurun_out/pmc_gemm2.log 2>&1
find gpurun_out/pmc_gemm* -name "*.csv"
