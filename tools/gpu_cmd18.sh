#!/bin/bash
# dense_x32 memory-bound test: dbg 16 (all blocks on one tile: operands L2-resident), 8 (no DMA), 4 (no epilogue)
set -u
for t in 6 8; do for d in 0 16 8 4; do echo "== fc tune $t dbg $d"; timeout -k 10 120 python tools/kbench.py --reps 5 --only fc_fwd,fc_dgrad --tune fc_fwd=$t,fc_dgrad=$t,stagger=$((512*d+2)) 2>&1 | grep -E "^fc" || exit 1; done; done
