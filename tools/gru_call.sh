#!/bin/bash
# GRU suite (persistence / fail-safe / recurrent tests) + whole-sequence timings + c5 line:
#   TAG=r04_x bash tools/gru_call.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG="${TAG:?set TAG}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "gru or recurrent or failsafe or rccl" > gpurun_out/${TAG}_t.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${TAG}_t.log | head; exit $rc; }
timeout -k 10 120 python -u tools/gru_bench.py --modes 0,1,3 > gpurun_out/${TAG}_g.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_g.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG LINES=c5 bash tools/lines_r04.sh
