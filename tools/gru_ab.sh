#!/bin/bash
# Same-box A/B of the whole-sequence GRU timings across library variants (LIBS, names
# under ppo-dash_amd/lib/libppo_hip_<name>.so; "cur" = libppo_hip.so), each checked
# bit-identical to the step launches:   TAG=x LIBS="cur loc0" bash tools/gru_ab.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
L=gpurun_out/${TAG:?set TAG}.log
for v in ${LIBS:-cur}; do
  lib=$PWD/ppo-dash_amd/lib/libppo_hip_$v.so; [ $v = cur ] && lib=$PWD/ppo-dash_amd/lib/libppo_hip.so
  echo "== $v" >> $L
  PPO_HIP_LIB=$lib timeout -k 10 120 python -u tools/gru_bench.py --modes 0,3 >> $L 2>&1 || { echo "rc=$? $v"; grep -v amdgpu.ids $L; exit 1; }
done
grep -v amdgpu.ids $L
