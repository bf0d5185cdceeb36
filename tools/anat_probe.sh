#!/bin/bash
# conv1 wgrad timing anatomy (dbg bits via stagger = 16*dbg + 2; wrong results by design):
# 1 skips the MFMAs, 2 the staging, 4 the DMAs, 8 the stagger.  Baseline kernels beside it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in ${DBGS:-0 1 2 3 4 5 6 7}; do
  echo "--- dbg=$d"
  timeout -k 10 120 python tools/kbench.py --B ${B:-65536} --reps 10 --only ${ONLY:-conv1_wgrad} --tune stagger=$((16*d + 2)) || exit $?
done
