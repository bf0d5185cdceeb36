#!/bin/bash
# Round-4 measurements in one GPU call: kbench A/B lines (tools/kb_lines.sh), the
# CU-contention probe (tools/cu_contention.py), then the targeted parity tests.
#   TAG=x bash tools/r04_probe.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
TAG="${TAG:?set TAG}"
mkdir -p gpurun_out
LINES="${LINES:---reps 10 --only conv2_fwd_mask,conv2_fwd|--reps 10 --only conv1_fwd_split,conv2_fwd_split,conv2_fwd_split_nm|--reps 10 --z1 256 --only conv1_wgrad --tune conv1_wgrad=7|--reps 10 --z1 256 --only conv1_wgrad --tune conv1_wgrad=8|--reps 10 --z1 256 --only conv1_wgrad}" \
  TESTK= bash tools/kb_lines.sh || exit $?
if [ "${CONTENTION:-1}" = 1 ]; then
  timeout -k 10 200 python -u tools/cu_contention.py > gpurun_out/${TAG}_cu.log 2>&1
  rc=$?; tail -1 gpurun_out/${TAG}_cu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -u tools/cu_contention.py --side-blocks 32 > gpurun_out/${TAG}_cu32.log 2>&1
  rc=$?; tail -1 gpurun_out/${TAG}_cu32.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "$TESTK" \
    > gpurun_out/${TAG}_t.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|Error" gpurun_out/${TAG}_t.log | tail -40; exit $rc
fi
