#!/bin/bash
# split-at-staging fc GEMM variants vs the defaults (kbench, c3 minibatch and rollout sizes)
set -e
mkdir -p gpurun_out
O=gpurun_out/ab_fc2.log
kb() { echo "== $*" >> $O; timeout -k 10 120 python -u tools/kbench.py "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for r in 1 2; do
  kb --reps 10 --only fc_fwd,fc_dgrad,fc_wgrad
  kb --reps 10 --only fc_fwd --tune fc_fwd=10
  kb --reps 10 --only fc_fwd --tune fc_fwd=11
  kb --reps 10 --only fc_fwd --tune fc_fwd=12
  kb --reps 10 --only fc_dgrad --tune fc_dgrad=10
  kb --reps 10 --only fc_dgrad --tune fc_dgrad=10,order=2
  kb --reps 10 --only fc_dgrad --tune fc_dgrad=11
  kb --reps 10 --only fc_wgrad --tune fc_wgrad=10
  kb --reps 10 --only fc_wgrad --tune fc_wgrad=10,order=2
  kb --reps 10 --only fc_wgrad --tune fc_wgrad=11
  kb --reps 10 --only fc_wgrad --tune fc_wgrad=11,order=2
done
kb --B 4096 --reps 20 --only fc_fwd
kb --B 4096 --reps 20 --only fc_fwd --tune fc_fwd=12
kb --B 4096 --reps 20 --only fc_fwd --tune fc_fwd=10
timeout -k 10 600 python -u -m pytest tests/test_dense.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dense.log 2>&1
