#!/bin/bash
# Build alternative libfm_hip.so variants with extra fm_pix.hip flags: tools/ab_build.sh NAME "-DFOO=1 ..."
# -> abvar/NAME/libfm_hip.so (git-ignored, travels to the GPU box) (select at run time with FM_HIP_LIB=...)
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -C "$ROOT/find_motion_amd/csrc" -j8 >/dev/null
D=$ROOT/abvar/$NAME; mkdir -p "$D"
HIPCC=/opt/rocm/bin/hipcc
$HIPCC -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -munsafe-fp-atomics $FLAGS \
  -c -x hip "$ROOT/find_motion_amd/csrc/fm_pix.hip" -o "$D/fm_pix.o"
O=$ROOT/build/fm_obj
$HIPCC -shared -fPIC --offload-arch=gfx950 -o "$D/libfm_hip.so" $O/fm_kernels.o $O/fm_fused.o "$D/fm_pix.o" $O/fm_ccl.o $O/fm_haar.o $O/fm_jpeg.o $O/fm_capi.o $O/fm_raster.o
echo "$D/libfm_hip.so"
