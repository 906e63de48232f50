# A/B of the fp64 GEMM's register-stage depth (VB_GEMM_STAGES): cold-operand
# GEMM chain micro-benchmark, then the config-4 step per library build.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do for S in 2 4 6 8; do
  echo "stages=$S"; timeout -k 5 60 ./scripts/ubench/gemm_chain_s$S 512
done; done 2>&1 | tee gpurun_out/gemm_stages.log
for i in 1 2; do for L in base s4 s6; do
  echo "lib=$L"; VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_$L.so timeout -k 5 120 python scripts/bench_fr.py --steps 40
done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/fr_stages.log
