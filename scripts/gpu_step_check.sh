set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  echo base; VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_base.so timeout -k 5 120 python scripts/bench_fr.py --steps 40
  echo new; timeout -k 5 120 python scripts/bench_fr.py --steps 40
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/fr_ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullrank.py tests/test_gpu_headline.py tests/test_gpu_vb.py tests/test_gpu_ia.py tests/test_gpu_wide.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
bash scripts/gpu_cfg5_prof.sh
