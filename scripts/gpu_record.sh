# Round GPU record on the current tree: config-4 A/B (base vs current build),
# the full -m gpu suite, the driver's bench command, a rocprofv3 kernel trace of
# that command (PASSES=trace of profile_r02.sh) and of the config-4 step.
# Every GPU step has its own limit; the first failure ends the script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -f viabel_amd/libviabel_amd_base.so ]; then
  for i in 1 2; do
    echo base; VIABEL_AMD_LIB=$PWD/viabel_amd/libviabel_amd_base.so timeout -k 5 120 python scripts/bench_fr.py --steps 40
    echo new; timeout -k 5 120 python scripts/bench_fr.py --steps 40
  done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/fr_ab.log
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
tail -c 600 gpurun_out/bench.log
PASSES=trace bash scripts/profile_r02.sh > /dev/null
bash scripts/gpu_fr_prof.sh
