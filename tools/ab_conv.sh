#!/bin/bash
# Same-box A/B of the conv kernels (KERNELS, kbench names): the current library
# against lib/libppo_hip_base.so (tools/build_base.sh REV), alternating, at the c3
# minibatch (Z = 256 splits); then the conv parity tests (TESTK) on the current one.
#   TAG=r04_x KERNELS=conv2_wgrad bash tools/ab_conv.sh -> gpurun_out/<TAG>_kb.log, <TAG>_t.log
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
TAG="${TAG:?set TAG}"
mkdir -p gpurun_out
L=gpurun_out/${TAG}_kb.log
K="${KERNELS:-conv1_fwd_mask,conv2_fwd_mask,conv2_wgrad,conv2_dgrad_bits,conv3_fwd,conv3_dgrad_bits,conv3_wgrad,conv1_wgrad}"
run() { echo "== $*" >> "$L"; timeout -k 10 200 "$@" >> "$L" 2>&1; rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc: $*"; tail -20 "$L"; exit $rc; }; }
for r in 1 2; do
  echo "== base" >> "$L"
  PPO_HIP_LIB=$PWD/ppo-dash_amd/lib/libppo_hip_base.so run python -u tools/kbench.py --reps 10 --z1 256 --z2 256 --only "$K"
  echo "== new" >> "$L"
  run python -u tools/kbench.py --reps 10 --z1 256 --z2 256 --only "$K"
done
grep -v amdgpu.ids "$L"
[ "${TESTK:-}" = none ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${TESTK:-conv or full_size or deterministic or engine_minibatch}" > gpurun_out/${TAG}_t.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/${TAG}_t.log; grep -E "FAILED|Error" gpurun_out/${TAG}_t.log | tail -20; tail -3 gpurun_out/${TAG}_t.log; exit $rc
