#!/bin/bash
set -e
mkdir -p gpurun_out
O=gpurun_out/ab_lin.log
for r in 1 2 3; do
  echo "== scalar" >> $O; timeout -k 10 120 python -u tools/kbench.py --reps 10 --only gru_in,gru_dx --tune fc_fwd=1,fc_dgrad=1 2>&1 | grep -v amdgpu.ids >> $O
  echo "== vector" >> $O; timeout -k 10 120 python -u tools/kbench.py --reps 10 --only gru_in,gru_dx 2>&1 | grep -v amdgpu.ids >> $O
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
timeout -k 10 600 python -u bench.py --recurrent --num-steps 256 --steps 3 --warmup 1 --no-cpu-baseline --no-gae-roofline --no-boundary > gpurun_out/b_c5.log 2>&1
