#!/bin/bash
# GPU box: conv2_dgrad tile sweep + PMC counter passes over the heavy trunk
# kernels (tools/kbench.py), each step under its own time limit.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
step() { local n=$1; shift; echo "== $n"; "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 20 "gpurun_out/$n.log"; [ $rc -ne 0 ] && exit $rc; return 0; }
step parity timeout -k 10 300 python -m pytest tests -m gpu -q -k "backward or full_iteration or golden"
for v in ${SWEEP:-0 1 2 3}; do
  step sweep_c2d_$v timeout -k 10 200 python tools/kbench.py --reps 5 --only conv2_dgrad --tune conv2_dgrad=$v
done
step kbench_all timeout -k 10 200 python tools/kbench.py --reps 5
if [ -n "${PMC:-}" ]; then
  ONLY="${ONLY:-conv1_fwd,conv1_wgrad,conv2_dgrad,conv3_dgrad,fc_fwd}" KB_ARGS="--reps 1" bash tools/pmc_passes.sh > gpurun_out/pmc.log 2>&1
  echo "pmc rc=$?"; tail -5 gpurun_out/pmc.log
fi
echo "== all done"
