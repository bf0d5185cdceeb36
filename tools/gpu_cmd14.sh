#!/bin/bash
# conv2 fwd x32 (tune 13): parity tests, then kbench A/B against 12
set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv2_fwd or conv2_mask" > gpurun_out/t14.log 2>&1; rc=$?; tail -3 gpurun_out/t14.log; [ $rc -eq 0 ] || exit $rc
for t in 12 13; do for d in 0 64; do echo "== conv2_fwd tune $t dbg $d"; timeout -k 10 120 python tools/kbench.py --reps 5 --only conv2_fwd_mask,conv2_fwd --tune conv2_fwd=$t,stagger=$((d+2)) 2>&1 | grep -E "^conv2" || exit 1; done; done
