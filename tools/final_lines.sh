#!/bin/bash
# end-of-session bench lines: c3 (driver default), --obs f32 / rgb, --half-precision
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/fin_c3.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 5 --obs f32 --no-cpu-baseline --no-gae-roofline --no-boundary > gpurun_out/fin_f32.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 5 --obs rgb --no-cpu-baseline --no-gae-roofline --no-boundary > gpurun_out/fin_rgb.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 5 --half-precision --no-cpu-baseline --no-gae-roofline --no-boundary > gpurun_out/fin_half.log 2>&1 || exit 1
