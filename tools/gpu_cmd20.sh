#!/bin/bash
set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k "persistent_bptt" -s > gpurun_out/t20.log 2>&1; tail -30 gpurun_out/t20.log | grep -E "mismatch|passed|failed"
