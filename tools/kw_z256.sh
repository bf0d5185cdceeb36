#!/bin/bash
# conv1 weight gradient variants at the engine's split (Z = 256) on the c3 minibatch;
# LIBS: library variants (cur = the in-tree build), TUNES: conv1_wgrad tune values
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do for L in ${LIBS:-cur}; do for t in ${TUNES:-8 9 10}; do
  if [ "$L" = cur ]; then unset PPO_HIP_LIB; else export PPO_HIP_LIB=ppo-dash_amd/lib/libppo_hip_$L.so; fi
  echo "--- lib $L tune $t z1 256"
  timeout -k 10 120 python tools/kbench.py --B 65536 --reps 10 --only conv1_wgrad --tune conv1_wgrad=$t --z1 256 2>&1 | grep -v amdgpu.ids || exit 1
done; done; done
