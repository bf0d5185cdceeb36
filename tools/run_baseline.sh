#!/bin/bash
# round-3 re-entry baseline: kernel micro-bench + c3 u8 / f32 bench lines
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/kbench.py --reps 5 --only conv1_fwd_mask,conv1_wgrad,conv1_fwd_f32,conv1_wgrad_f32,conv1_fwd_rgb,conv1_wgrad_rgb,conv2_fwd_mask,conv2_wgrad,conv2_dgrad_bits,fc_fwd,fc_dgrad,fc_wgrad > gpurun_out/kb0.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/b0_u8.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --obs f32 --no-cpu-baseline --no-gae-roofline --no-boundary > gpurun_out/b0_f32.log 2>&1
