#!/bin/bash
set -u
timeout -k 10 400 python -u -m pytest tests/test_small_batch.py tests/test_evaluation.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t24.log 2>&1; rc=$?; tail -3 gpurun_out/t24.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/eval_probe.py
