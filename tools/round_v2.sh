#!/bin/bash
# obs tests for the preprocess change, the f32 bench line, then the round profile set
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_obs_boundary.py tests/test_obs_paths.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_obs.log 2>&1 || { tail -20 gpurun_out/t_obs.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --obs f32 --no-cpu-baseline --no-gae-roofline --no-boundary > gpurun_out/b_f32.log 2>&1 || exit 1
KERNEL_REGEX=conv2_fwd_x9c bash tools/profile_round.sh
