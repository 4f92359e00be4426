#!/bin/bash
# Build a libfm_hip.so variant with extra flags on ONE source file: tools/ab_build_file.sh NAME fm_ccl.hip "-DFOO=1 ..."
# -> abvar/NAME/libfm_hip.so (git-ignored, travels to the GPU box; select with FM_HIP_LIB=...)
set -e
NAME=$1; SRC=$2; FLAGS=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -C "$ROOT/find_motion_amd/csrc" -j8 >/dev/null
D=$ROOT/abvar/$NAME; mkdir -p "$D"
HIPCC=/opt/rocm/bin/hipcc
B=$(basename "$SRC" .hip); B=$(basename "$B" .cpp)
$HIPCC -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -munsafe-fp-atomics $FLAGS \
  -c -x hip "$ROOT/find_motion_amd/csrc/$SRC" -o "$D/$B.o"
O=$ROOT/build/fm_obj
OBJS=""
for o in fm_kernels fm_fused fm_pix fm_ccl fm_haar fm_jpeg fm_capi fm_raster; do
  if [ "$o" = "$B" ]; then OBJS="$OBJS $D/$B.o"; else OBJS="$OBJS $O/$o.o"; fi
done
$HIPCC -shared -fPIC --offload-arch=gfx950 -o "$D/libfm_hip.so" $OBJS
echo "$D/libfm_hip.so"
