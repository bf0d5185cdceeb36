#!/bin/bash
# new c5 4096-lane rollout test, then conv1f anatomy (fp32 rows)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_full_size.py -k rollout_4096 -x -v -s --timeout 250 --timeout-method thread > gpurun_out/t27.log 2>&1; rc=$?; tail -3 gpurun_out/t27.log; [ $rc -eq 0 ] || exit $rc
ONLY=conv1_fwd_f32,conv1_wgrad_f32,conv1_fwd_mask,conv1_wgrad DBGS="0 1 2 4 8" bash tools/anat_c1f.sh > gpurun_out/anat27.log 2>&1; rc=$?; cat gpurun_out/anat27.log | grep -v "^$" | tail -40; exit $rc
