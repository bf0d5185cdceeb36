#!/bin/bash
set -e
mkdir -p gpurun_out
O=gpurun_out/ab_fcw.log
for r in 1 2 3; do
  echo "== scalar" >> $O; timeout -k 10 120 python -u tools/kbench.py --reps 10 --only fc_wgrad --tune order=3 2>&1 | grep -v amdgpu.ids >> $O
  echo "== vector" >> $O; timeout -k 10 120 python -u tools/kbench.py --reps 10 --only fc_wgrad 2>&1 | grep -v amdgpu.ids >> $O
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
