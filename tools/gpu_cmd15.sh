#!/bin/bash
# conv2 fwd x9c staging anatomy: 128 no split (same traffic), 256 no LDS put (loads kept), 64 no staging
set -u
for d in 0 128 256 64; do echo "== conv2_fwd dbg $d"; timeout -k 10 120 python tools/kbench.py --reps 5 --only conv2_fwd_mask --tune stagger=$((d+2)) 2>&1 | grep -E "^conv2" || exit 1; done
