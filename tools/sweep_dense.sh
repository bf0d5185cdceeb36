#!/bin/bash
# GPU box: tile-shape sweep of the GEMM core on fc forward (dense, K=1568) and
# conv2 forward (implicit GEMM, N=64).  One process per setting.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in ${FC:-0 1 2 3 4 5}; do
  echo "--- fc_fwd variant $v"
  timeout -k 10 120 python tools/kbench.py --reps 10 --only fc_fwd --tune fc_fwd=$v || exit $?
done
for v in ${C2:-0 3 4 5 6}; do
  echo "--- conv2_fwd variant $v"
  timeout -k 10 120 python tools/kbench.py --reps 10 --only conv2_fwd --tune conv2_fwd=$v || exit $?
done
echo done
