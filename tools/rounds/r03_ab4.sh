#!/bin/bash
ROUNDS="1 2 3" tools/ab_steady.sh p5_base p5_even p5_hs p5_both
