#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_obs_boundary.py tests/test_obs_paths.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_obs.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --obs f32 --no-cpu-baseline --no-gae-roofline > gpurun_out/b_f32.log 2>&1
