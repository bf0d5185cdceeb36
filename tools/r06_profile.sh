#!/bin/bash
# Round-6 profile set (GPU box): tools/profile_round.sh (bench line, rocprofv3
# kernel stats, FETCH / WRITE passes of the dominant kernel, the MFMA pass with
# GRBM_GUI_ACTIVE for the shader clock), then the c5 line.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
KERNEL_REGEX="conv2_fwd_x9c_kernel|conv2_fwd_lone_kernel" timeout -k 10 1000 bash tools/profile_round.sh || exit $?
timeout -k 10 600 python -u bench.py --recurrent --num-steps 256 --no-cpu-baseline --no-gae-roofline --no-boundary > gpurun_out/r06_c5_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r06_c5_bench.log | cut -c1-300; exit $rc
