#!/bin/bash
# GPU suite + smoke + c3 bench line, every log under a unique per-call name:
#   TAG=r04_a bash tools/gpu_suite.sh        -> gpurun_out/<TAG>_{tests,smoke,bench}.log
# Set SUITE=0 to skip the test suite, BENCH=0 to skip the bench, K="-k expr" to
# select tests.  Stops at the first failing step (no GPU step after a failure).
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
TAG="${TAG:?set TAG}"
mkdir -p gpurun_out
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:-} > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 500 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1
  rc=$?; grep '^{' gpurun_out/${TAG}_bench.log | cut -c1-400; exit $rc
fi
