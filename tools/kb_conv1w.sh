#!/bin/bash
# conv1 wgrad A/B at the engine's split count (one block per CU): variants x dbg anatomy
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
Z=${Z:-256}
for v in ${VARIANTS:-3 4 5}; do
  for d in ${DBGS:-0}; do
    echo "--- variant=$v dbg=$d z1=$Z"
    timeout -k 10 120 python tools/kbench.py --B ${B:-65536} --reps 10 --z1 $Z --only conv1_wgrad --tune conv1_wgrad=$v,stagger=$((16*d + 2)) || exit $?
  done
done
