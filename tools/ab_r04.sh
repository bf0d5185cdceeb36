#!/bin/bash
# Round-4 kernel A/B on one box (kbench at the c3 minibatch, 65,536 images; the
# engine's split counts Z = 256): the fp32-a1 conv1 -> conv2 kernels against the
# pre-split hand-off (a1split.hip), and the part-pipelined conv1 weight gradient
# (tune 5) against the k-split kernel (conv1w.hip, tune 7); then their parity tests.
#   TAG=r04_ab bash tools/ab_r04.sh   -> gpurun_out/<TAG>_kb.log, <TAG>_t.log
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
TAG="${TAG:?set TAG}"
mkdir -p gpurun_out
L=gpurun_out/${TAG}_kb.log
run() { echo "== $*" >> "$L"; timeout -k 10 200 "$@" >> "$L" 2>&1; rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc: $*"; tail -20 "$L"; exit $rc; }; }
for r in 1 2; do
  run python -u tools/kbench.py --reps 10 --z1 256 --z2 256 --only conv1_fwd_mask,conv2_fwd_mask,conv2_fwd,conv2_wgrad,conv1_wgrad
  run python -u tools/kbench.py --reps 10 --z2 256 --only conv1_fwd_split,conv2_fwd_split,conv2_fwd_split_nm,conv2_wgrad_split
  run python -u tools/kbench.py --reps 10 --z1 256 --only conv1_wgrad --tune conv1_wgrad=7
done
run python -u tools/kbench.py --B 4096 --reps 20 --only conv1_fwd,conv2_fwd,conv1_fwd_split,conv2_fwd_split_nm
cat "$L"
timeout -k 10 600 python -u -m pytest tests/test_a1split.py tests/test_gpu_parity.py tests/test_half.py -x -v \
  --timeout 120 --timeout-method thread -k "a1split or split_equals or conv1_split or engine_minibatch or conv1_wgrad_variants or deterministic" \
  > gpurun_out/${TAG}_t.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_t.log; exit $rc
