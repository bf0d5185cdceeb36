#!/bin/bash
# c5 (GRU H=256 + 14 vector obs, 4096 x 256) bench line and rocprof kernel stats
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --recurrent --num-steps 256 --steps 3 --warmup 1 --no-cpu-baseline --no-gae-roofline --no-boundary > gpurun_out/b_c5.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o run -- python3 bench.py --recurrent --num-steps 256 --steps 2 --warmup 1 --no-cpu-baseline --no-gae-roofline --no-boundary --no-profile-pass > gpurun_out/b_c5_prof.log 2>&1
