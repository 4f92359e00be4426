#!/bin/bash
# Build an alternative libfm_hip.so with extra flags on some sources, for A/B runs on the GPU box:
#   tools/ab_build.sh NAME "-DFOO=1 ..." [fm_pix fm_ccl ...]   (default: every source)
# -> abvar/NAME/libfm_hip.so (git-ignored, travels with the tree); select it with FM_HIP_LIB=...
set -e
NAME=$1; FLAGS=$2; shift 2
SRCS=${*:-fm_kernels fm_fused fm_pix fm_small fm_ccl fm_haar fm_jpeg fm_capi}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -C "$ROOT/find_motion_amd/csrc" -j8 >/dev/null
D=$ROOT/abvar/$NAME; mkdir -p "$D"
HIPCC=/opt/rocm/bin/hipcc
O=$ROOT/build/fm_obj
OBJS=""
for s in fm_kernels fm_fused fm_pix fm_small fm_ccl fm_haar fm_jpeg fm_capi; do
  if [[ " $SRCS " == *" $s "* ]]; then
    src=$ROOT/find_motion_amd/csrc/$s.hip; [ -f "$src" ] || src=$ROOT/find_motion_amd/csrc/$s.cpp
    $HIPCC -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -munsafe-fp-atomics $FLAGS \
      -c -x hip "$src" -o "$D/$s.o" &
    PIDS="$PIDS $!"
    OBJS="$OBJS $D/$s.o"
  else
    OBJS="$OBJS $O/$s.o"
  fi
done
for p in $PIDS; do wait "$p" || { echo "ab_build: a compile failed" >&2; exit 1; }; done
$HIPCC -shared -fPIC --offload-arch=gfx950 -o "$D/libfm_hip.so" $OBJS $O/fm_raster.o
echo "$D/libfm_hip.so"
