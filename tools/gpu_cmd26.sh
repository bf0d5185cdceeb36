#!/bin/bash
# half-precision tests (verbose, printed errors), then the full GPU suite + smoke
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_half.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/half.log 2>&1; rc=$?; tail -5 gpurun_out/half.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_full.sh
