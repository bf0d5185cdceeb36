#!/bin/bash
# A/B of two library builds on the fc GEMMs (kbench), alternating
set -e
mkdir -p gpurun_out
L=ppo-dash_amd/lib/ab
for r in 1 2; do
  for v in old new; do
    echo "== $v B=65536" >> gpurun_out/ab_fc.log
    PPO_HIP_LIB=$L/$v.so timeout -k 10 120 python -u tools/kbench.py --reps 10 --only fc_fwd,fc_dgrad,fc_wgrad,conv3_wgrad >> gpurun_out/ab_fc.log 2>&1
    echo "== $v B=4096" >> gpurun_out/ab_fc.log
    PPO_HIP_LIB=$L/$v.so timeout -k 10 120 python -u tools/kbench.py --B 4096 --reps 20 --only fc_fwd >> gpurun_out/ab_fc.log 2>&1
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "linear or fc or dense or wgrad or mlp or gru or full_size" > gpurun_out/t_fc.log 2>&1
