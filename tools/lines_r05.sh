#!/bin/bash
# Secondary bench lines (c5 recurrent, RGB / fp32 observations, half precision):
#   TAG=r05_zb bash tools/lines_r05.sh -> gpurun_out/<TAG>_{c5,rgb,f32,half}.json
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG="${TAG:?set TAG}"
run() { name=$1; shift; timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-gae-roofline --no-boundary "$@" > gpurun_out/${TAG}_$name.log 2>&1 || { tail -5 gpurun_out/${TAG}_$name.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_$name.log | tail -1 > gpurun_out/${TAG}_$name.json
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
run c5 --recurrent --num-steps 256
run rgb --obs rgb
run f32 --obs f32
run half --half-precision
