#!/bin/bash
# Build the whole library with extra compile flags into
# viabel_amd/libviabel_amd_<name>.so (A/B experiments; select it at run time
# with VIABEL_AMD_LIB).   bash scripts/build_variant.sh base "-DVB_GEMM_KTG=32 -DVB_GEMM_GS=4"
set -e
name=$1; flags=$2
cd "$(dirname "$0")/../viabel_amd/csrc"
mkdir -p build/var_$name
hash=$(make -s print-hash)
objs=""
for f in vb_mf vb_fr vb_rhat vb_bounds vb_psis vb_probe vb_capi; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $flags \
    "-DVB_SRC_HASH=\"$hash\"" -c $f.hip -o build/var_$name/$f.o &
  objs="$objs build/var_$name/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libviabel_amd_$name.so $objs -lrocsolver -lrocblas
echo built ../libviabel_amd_$name.so
