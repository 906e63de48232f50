set -u
mkdir -p gpurun_out/kw2
LIBS="nokw kw" ROUNDS=3 timeout -k 10 300 bash scripts/gpu_ab_headline.sh > gpurun_out/kw2/headline.log 2>&1 &&
LIBS="viabel_amd/libviabel_amd_nokw.so viabel_amd/libviabel_amd_kw.so" ROUNDS_OUT=2 timeout -k 10 300 bash scripts/ab_block.sh > gpurun_out/kw2/block.log 2>&1 &&
LIBS="nokw kw" ROUNDS=2 timeout -k 10 200 bash scripts/gpu_ab_fr2.sh > gpurun_out/kw2/cfg4.log 2>&1
