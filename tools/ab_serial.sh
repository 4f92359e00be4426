#!/bin/bash
# Serial-mode (contour pass on the pixel stream) pixel-kernel A/B of fm_pix.hip flag variants.
# Build here:  tools/ab_serial.sh build NAME "-DFLAG=.." [NAME "-D.." ...]
# GPU box:     tools/ab_serial.sh run NAME [NAME ...]      (alternating, 2 rounds)
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
MODE=$1; shift
if [ "$MODE" = build ]; then
  make -C "$ROOT/find_motion_amd/csrc" -j8 >/dev/null; make -C "$ROOT/find_motion_amd/csrc" -j8 VARIANT=dev >/dev/null
  while [ $# -gt 0 ]; do
    N=$1; F=$2; shift 2
    D=$ROOT/abvar/s_$N; mkdir -p "$D"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -munsafe-fp-atomics \
      $F -c -x hip "$ROOT/find_motion_amd/csrc/fm_pix.hip" -o "$D/fm_pix.o"
    O=$ROOT/build/fm_obj; OD=$ROOT/build/fm_obj_dev
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$D/libfm_hip.so" $O/fm_kernels.o $O/fm_fused.o "$D/fm_pix.o" \
      $O/fm_ccl.o $O/fm_haar.o $OD/fm_capi.o $O/fm_raster.o
    rm -f "$D/fm_pix.o"
  done
  exit 0
fi
for r in 1 2; do
  for N in "$@"; do
    FM_HIP_LIB=$ROOT/abvar/s_$N/libfm_hip.so FM_SERIAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed --steps 30 \
      | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$N round $r', d['value'], d['roofline']['avg_launch_us'])"
  done
done
