#!/bin/bash
for D in abvar/*/; do echo "== $D"; FM_HIP_LIB=$PWD/$D/libfm_hip.so timeout -k 10 120 python tools/dbg_mask.py 2>&1 | grep frame; done
