# Config-4 A/B, interleaved: libviabel_amd_base.so (before), libviabel_amd.so
# (after), optional libviabel_amd_$ALT.so; cold-operand GEMM chain builds
# scripts/ubench/gemm_chain_bm{32,16}; full-rank / headline parity tests on the
# default build and on the ALT build; kernel trace of the default build.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ALT=${ALT:-bm16}
for i in 1 2; do for B in 32 16; do
  [ -x ./scripts/ubench/gemm_chain_bm$B ] && { echo "bm=$B"; timeout -k 5 60 ./scripts/ubench/gemm_chain_bm$B 512; }
done; done 2>&1 | tee gpurun_out/gemm_bm.log
for i in 1 2 3; do
  for L in base "" $ALT; do
    lib=$PWD/viabel_amd/libviabel_amd${L:+_$L}.so
    [ -f $lib ] || continue
    echo "lib=${L:-new}"; VIABEL_AMD_LIB=$lib timeout -k 5 120 python scripts/bench_fr.py --steps 40
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/fr_ab.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_headline.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
if [ -f viabel_amd/libviabel_amd_$ALT.so ]; then
  VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_$ALT.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_headline.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
fi
bash scripts/gpu_fr_prof.sh
