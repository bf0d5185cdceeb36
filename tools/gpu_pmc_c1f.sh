#!/bin/bash
# PMC passes (SQ counters) of the conv1f kernels through kbench, then a per-kernel summary
set -u
ONLY=${ONLY:-conv1_fwd_f32,conv1_wgrad_f32} TUNE="stagger=2" bash tools/pmc_sq.sh > gpurun_out/pmc_c1f.log 2>&1 || { tail -20 gpurun_out/pmc_c1f.log; exit 1; }
for k in conv1_fwd_x6w_kernel conv1_wgrad_x6_kernel; do echo "== $k"; python tools/pmc_parse.py "$k" gpurun_out/pmc1; done
