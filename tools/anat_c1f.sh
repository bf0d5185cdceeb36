#!/bin/bash
# Timing anatomy of the conv1f.hip kernels (kbench, minibatch 65,536): default,
# then each dbg skip flag (stagger = 16 * dbg; results are wrong by design).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
K="${ONLY:-conv1_fwd_f32,conv1_fwd_rgb,conv1_wgrad_f32,conv1_wgrad_rgb,conv1_fwd_mask,conv1_wgrad}"
for d in ${DBGS:-0 1 2 4 8 16}; do
  echo "== dbg $d"
  timeout -k 10 300 python tools/kbench.py --reps 3 --only "$K" --tune "stagger=$((16 * d + 2))" || exit $?
done
