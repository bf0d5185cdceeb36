#!/bin/bash
# the --obs rgb forward (affine fold, rgbaff.hip): its tests, a same-box kbench A/B
# against lib/libppo_hip_base.so, and the rgb bench line
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T="${TAG:-r04_rgb}"
timeout -k 10 400 python -u -m pytest tests/test_obs_paths.py tests/test_full_size.py -x -v --timeout 120 --timeout-method thread -k "rgb or fused or obs_paths or float_obs" > gpurun_out/${T}_t.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/${T}_t.log; grep -E "FAILED|Error|assert" gpurun_out/${T}_t.log | head -10; tail -2 gpurun_out/${T}_t.log; [ $rc -eq 0 ] || exit $rc
TAG=$T KERNELS=${KERNELS:-conv1_fwd_rgb,conv1_wgrad_rgb} TESTK=none bash tools/ab_conv.sh || exit 1
TAG=$T LINES="rgb" bash tools/lines_r04.sh
