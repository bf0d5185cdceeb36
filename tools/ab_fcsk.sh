#!/bin/bash
set -e
mkdir -p gpurun_out
O=gpurun_out/ab_fcsk.log
kb() { echo "== $*" >> $O; timeout -k 10 120 python -u tools/kbench.py "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for r in 1 2; do
  kb --B 4096 --reps 50 --only fc_fwd
  kb --B 4096 --reps 50 --only fc_fwd_ws --tune fc_splitk=2
  kb --B 4096 --reps 50 --only fc_fwd_ws --tune fc_splitk=3
  kb --B 4096 --reps 50 --only fc_fwd_ws --tune fc_splitk=4
done
timeout -k 10 300 python -u -m pytest tests/test_dense.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dense.log 2>&1
