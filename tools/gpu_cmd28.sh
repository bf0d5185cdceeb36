#!/bin/bash
# conv1f anatomy, combined skip flags (fp32 rows): 6 = compute+epilogue only, 14 = compute only, 3 = loads+epi, 5 = put+epi
set -u
mkdir -p gpurun_out
ONLY=conv1_fwd_f32,conv1_wgrad_f32 DBGS="6 14 3 5 13 11" bash tools/anat_c1f.sh > gpurun_out/anat28.log 2>&1; rc=$?; grep -v "^$\|amdgpu.ids" gpurun_out/anat28.log | tail -40; exit $rc
