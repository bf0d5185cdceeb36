#!/bin/bash
# dense_x32 timing anatomy (stagger bits 512 no MFMA, 1024 no split, 2048 no epilogue, 4096 no DMA) + SQ counters
set -u
for d in 0 1 2 4 8 3 9; do echo "== dense dbg $d"; timeout -k 10 120 python tools/kbench.py --reps 5 --only fc_fwd,fc_dgrad --tune fc_fwd=6,fc_dgrad=6,stagger=$((512*d+2)) 2>&1 | grep -E "^fc" || exit 1; done
ONLY=fc_fwd TUNE="fc_fwd=6,stagger=2" bash tools/pmc_sq.sh > gpurun_out/pmc_dense.log 2>&1 || { tail -20 gpurun_out/pmc_dense.log; exit 1; }
python tools/pmc_parse.py dense_x32 gpurun_out/pmc1
