#!/bin/bash
# Full GPU suite + smoke + c3 bench line (tools/gpu_suite.sh), then the whole-sequence
# GRU timings per persist mode and the c5 line (tools/lines_r04.sh):
#   TAG=r05_x bash tools/suite_gru.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG="${TAG:?set TAG}"
TAG=$TAG bash tools/gpu_suite.sh || exit $?
timeout -k 10 120 python -u tools/gru_bench.py --modes 0,1,3 > gpurun_out/${TAG}_g.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${TAG}_g.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG LINES=c5 bash tools/lines_r04.sh
