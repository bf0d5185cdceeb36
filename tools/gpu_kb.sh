#!/bin/bash
# kbench A/B of tune variants: KB="name:tune[,tune]|..." entries, B sizes in BS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BS="${BS:-65536 4096}"
IFS='|' read -ra ENTRIES <<< "$KB"
LIBS="${LIBS:-cur}"
for B in $BS; do
  for e in "${ENTRIES[@]}"; do
    only=${e%%:*}; tune=${e#*:}
    for L in $LIBS; do
      if [ "$L" = cur ]; then unset PPO_HIP_LIB; else export PPO_HIP_LIB=ppo-dash_amd/lib/libppo_hip_$L.so; fi
      echo "--- B=$B lib=$L only=$only tune=$tune"
      timeout -k 10 120 python tools/kbench.py --B $B --reps 10 --only "$only" --tune "$tune"
      rc=$?; if [ $rc -ne 0 ]; then echo "!! rc=$rc"; exit $rc; fi
    done
  done
done
