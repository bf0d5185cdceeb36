#!/bin/bash
# fc GEMMs on dense_x32 (tune 6: BK 32 x 2 stages, 7: BK 16 x 4 stages): parity, then kbench A/B
set -u
timeout -k 10 300 python -u -m pytest tests/test_dense.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t16.log 2>&1; rc=$?; tail -3 gpurun_out/t16.log; [ $rc -eq 0 ] || exit $rc
for t in 0 6 7 8; do echo "== fc tune $t"; timeout -k 10 120 python tools/kbench.py --reps 5 --only fc_fwd,fc_dgrad --tune fc_fwd=$t,fc_dgrad=$t 2>&1 | grep -E "^fc" || exit 1; done

