#!/bin/bash
# conv2 wgrad half-staged (tune 9): parity + bit-identity, kbench A/B
set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv2_wgrad" > gpurun_out/t22.log 2>&1; rc=$?; tail -3 gpurun_out/t22.log; [ $rc -eq 0 ] || exit $rc
for t in 8 9 8 9; do echo "== conv2_wgrad tune $t"; timeout -k 10 120 python tools/kbench.py --reps 5 --only conv2_wgrad --tune conv2_wgrad=$t 2>&1 | grep -E "^conv2" || exit 1; done
