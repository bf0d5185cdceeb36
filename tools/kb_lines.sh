#!/bin/bash
# kbench A/B lines on one box: LINES="args1|args2|..." (each a tools/kbench.py argument
# list), run REPS_AB (default 2) times alternating; then optional pytest -k "$TESTK".
#   TAG=x LINES="--only conv2_fwd_mask|--only conv2_fwd_split" bash tools/kb_lines.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
TAG="${TAG:?set TAG}"
mkdir -p gpurun_out
L=gpurun_out/${TAG}_kb.log
IFS='|' read -ra ARGS <<< "${LINES:?set LINES}"
for r in $(seq 1 "${REPS_AB:-2}"); do
  for a in "${ARGS[@]}"; do
    echo "== $a" >> "$L"
    timeout -k 10 200 python -u tools/kbench.py $a >> "$L" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc: $a"; tail -20 "$L"; exit $rc; }
  done
done
grep -v amdgpu.ids "$L"
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$TESTK" \
    > gpurun_out/${TAG}_t.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|Error" gpurun_out/${TAG}_t.log | tail -30; exit $rc
fi
