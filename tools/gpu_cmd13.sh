#!/bin/bash
# timing anatomy of the conv2 kernels (stagger dbg bits: 16 no MFMA, 32 no epilogue, 64 no staging)
set -u
for op in conv2_fwd_mask conv2_wgrad conv2_dgrad_bits; do
  for d in 0 16 32 64 80; do
    echo "== $op dbg $d"; timeout -k 10 120 python tools/kbench.py --reps 5 --only $op --tune stagger=$((d+2)) 2>&1 | grep -E "^$op" || exit 1
  done
done
