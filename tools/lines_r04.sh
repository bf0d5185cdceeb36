#!/bin/bash
# The secondary bench lines (c5, --obs f32 / rgb, --half-precision) on one box:
#   TAG=x bash tools/lines_r04.sh   -> gpurun_out/<TAG>_{c5,f32,rgb,half}.log
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
TAG="${TAG:?set TAG}"
mkdir -p gpurun_out
NB="--no-cpu-baseline --no-gae-roofline --no-boundary"
run() { local name=$1; shift; timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${TAG}_${name}.log 2>&1; rc=$?;
        grep '^{' gpurun_out/${TAG}_${name}.log | cut -c1-330; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_${name}.log; exit $rc; }; }
for l in ${LINES:-c5 f32 rgb half}; do
  case $l in
    c5) run c5 --recurrent --num-steps 256 --steps 3 --warmup 1 $NB ;;
    f32) run f32 --steps 5 --obs f32 $NB ;;
    rgb) run rgb --steps 5 --obs rgb $NB ;;
    half) run half --steps 5 --half-precision $NB ;;
  esac
done
