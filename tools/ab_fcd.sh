#!/bin/bash
set -e
mkdir -p gpurun_out
O=gpurun_out/ab_fcd.log
for r in 1 2 3; do
  echo "== scalar epilogues" >> $O; timeout -k 10 120 python -u tools/kbench.py --reps 10 --only fc_fwd,fc_dgrad --tune fc_dgrad=1,fc_fwd=1 2>&1 | grep -v amdgpu.ids >> $O
  echo "== vector epilogues" >> $O; timeout -k 10 120 python -u tools/kbench.py --reps 10 --only fc_fwd,fc_dgrad 2>&1 | grep -v amdgpu.ids >> $O
done
timeout -k 10 300 python -u -m pytest tests/test_dense.py tests/test_small_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dense.log 2>&1
