#!/bin/bash
set -e
mkdir -p gpurun_out
O=gpurun_out/ab_heads.log
for r in 1 2 3; do for v in old new; do
  echo "== $v" >> $O
  PPO_HIP_LIB=ppo-dash_amd/lib/ab/$v.so timeout -k 10 120 python -u tools/kbench.py --B 4096 --reps 100 --only heads_act 2>&1 | grep -v amdgpu.ids >> $O
done; done
