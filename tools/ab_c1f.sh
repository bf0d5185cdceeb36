#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_obs_paths.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_c1f.log 2>&1
O=gpurun_out/ab_c1f.log
for r in 1 2; do
  echo "== default" >> $O; timeout -k 10 120 python -u tools/kbench.py --reps 10 --only conv1_fwd_f32 2>&1 | grep -v amdgpu.ids >> $O
  echo "== tune 7" >> $O; timeout -k 10 120 python -u tools/kbench.py --reps 10 --only conv1_fwd_f32 --tune conv1_fwd=7 2>&1 | grep -v amdgpu.ids >> $O
done
