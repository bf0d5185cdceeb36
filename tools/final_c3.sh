#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/fin2_c3.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6 -o run -- python3 bench.py --no-cpu-baseline --no-gae-roofline --no-boundary --steps 5 > gpurun_out/fin2_prof.log 2>&1
