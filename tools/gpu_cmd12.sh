#!/bin/bash
# SQ anatomy of the conv trunk kernels (conv2 fwd / dgrad / wgrad, conv3 fwd) + kbench times
set -u
timeout -k 10 300 python tools/kbench.py --reps 5 --only conv2_fwd_mask,conv2_dgrad_bits,conv2_wgrad,conv3_fwd,conv3_dgrad_bits,conv3_wgrad 2>&1 | grep -v amdgpu || exit 1
ONLY=conv2_fwd_mask,conv2_dgrad_bits,conv2_wgrad,conv3_fwd TUNE="stagger=2" bash tools/pmc_sq.sh > gpurun_out/pmc_trunk.log 2>&1 || { tail -20 gpurun_out/pmc_trunk.log; exit 1; }
for k in conv2_fwd_x9c conv2_dgrad_x9 conv2_wgrad_x9 conv3_fwd_x9; do echo "== $k"; python tools/pmc_parse.py "$k" gpurun_out/pmc1; done
