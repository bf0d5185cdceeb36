#!/bin/bash
# tile-variant sweep of the heavy GEMMs (one process per setting; GPU box only)
cd "${GRAFT_REPO_ROOT:-.}"
for v in 0 1 2 3 4; do
  echo "--- N32 variant $v"
  timeout -k 10 200 python tools/kbench.py --reps 5 --only conv1_fwd,conv3_fwd,conv2_dgrad \
      --tune conv1_fwd=$v,conv3_fwd=$v,conv2_dgrad=$v || exit $?
done
for v in 0 1 2; do
  echo "--- N64 variant $v"
  timeout -k 10 200 python tools/kbench.py --reps 5 --only conv3_dgrad --tune conv3_dgrad=$v || exit $?
done
for v in 0 1; do
  echo "--- conv1_wgrad variant $v"
  timeout -k 10 200 python tools/kbench.py --reps 5 --only conv1_wgrad,conv1_wreduce --tune conv1_wgrad=$v || exit $?
done
echo "--- all"
timeout -k 10 200 python tools/kbench.py --reps 5
