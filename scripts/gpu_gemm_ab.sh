# GEMM A/B: cold-operand chain (committed header: gemm_chain_old, experiment:
# gemm_chain_exp), then config 4 with libviabel_amd_base.so vs libviabel_amd_exp.so,
# then the full-rank / headline / bounds / notebook parity tests on the
# experiment library.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  echo old; timeout -k 5 60 ./scripts/ubench/gemm_chain_old 512
  echo exp; timeout -k 5 60 ./scripts/ubench/gemm_chain_exp 512
done 2>&1 | tee gpurun_out/gemm_ab.log
for i in 1 2 3; do
  echo cur; VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_base.so timeout -k 5 120 python scripts/bench_fr.py --steps 40
  echo exp; VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_exp.so timeout -k 5 120 python scripts/bench_fr.py --steps 40
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/fr_ab.log
VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_exp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_headline.py tests/test_gpu_bounds_psis.py tests/test_gpu_notebooks.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
