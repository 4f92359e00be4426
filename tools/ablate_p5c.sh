#!/bin/bash
# k_pix5 stage ablations with the skip fixed at compile time (the product kernel's code shape), serial
# contour pass (dev-build fm_capi for FM_SERIAL).  Build here first: tools/ablate_p5c.sh build "0 1 2 4 8"
# then on the GPU box: tools/ablate_p5c.sh run "0 1 2 4 8".  Bits: 1 gray, 2 chain, 4 loads, 8 taps.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
MODE=$1; SKIPS=${2:-"0 1 2 4 8"}
if [ "$MODE" = build ]; then
  make -C "$ROOT/find_motion_amd/csrc" -j8 >/dev/null; make -C "$ROOT/find_motion_amd/csrc" -j8 VARIANT=dev >/dev/null
  for sk in $SKIPS; do
    D=$ROOT/abvar/p5s$sk; mkdir -p "$D"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -munsafe-fp-atomics \
      -DFM_P5_SKIP=$sk -c -x hip "$ROOT/find_motion_amd/csrc/fm_pix.hip" -o "$D/fm_pix.o"
    O=$ROOT/build/fm_obj; OD=$ROOT/build/fm_obj_dev
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$D/libfm_hip.so" $O/fm_kernels.o $O/fm_fused.o "$D/fm_pix.o" \
      $O/fm_ccl.o $O/fm_haar.o $OD/fm_capi.o $O/fm_raster.o
  done
  exit 0
fi
for sk in $SKIPS; do
  FM_HIP_LIB=$ROOT/abvar/p5s$sk/libfm_hip.so FM_SERIAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-fed --steps 30 \
    | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('skip $sk', d['roofline']['avg_launch_us'])"
done
