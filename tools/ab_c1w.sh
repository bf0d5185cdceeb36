#!/bin/bash
set -e
mkdir -p gpurun_out
O=gpurun_out/ab_c1w.log
kb() { echo "== $*" >> $O; timeout -k 10 120 python -u tools/kbench.py "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for r in 1 2 3; do
  kb --reps 10 --only conv1_wgrad --tune conv1_wgrad=5
  kb --reps 10 --only conv1_wgrad --tune conv1_wgrad=7
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "conv1_wgrad" > gpurun_out/t_c1w.log 2>&1
