# Config-4 A/B: libviabel_amd_base.so (before) vs libviabel_amd.so (after),
# interleaved, then the full-rank parity tests and a kernel trace of the new build.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  echo base; VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_base.so timeout -k 5 120 python scripts/bench_fr.py --steps 40
  echo new; timeout -k 5 120 python scripts/bench_fr.py --steps 40
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/fr_ab.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_headline.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
bash scripts/gpu_fr_prof.sh
