#!/bin/bash
export ARGS="--width 3840 --height 2160 --blur-scale 183 --streams 4 --batch 64 --ring 64 --ring-period 16 --steps 10 --warmup 3"
ROUNDS="1 2" tools/ab_shape.sh pw_a pw_valu pw_split pw_vs
