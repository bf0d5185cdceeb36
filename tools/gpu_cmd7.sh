timeout -k 10 600 python -u -m pytest tests/test_obs_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_obs.log 2>&1; tail -3 gpurun_out/t_obs.log
ONLY=conv1_fwd_f32,conv1_fwd_rgb,conv1_wgrad_f32,conv1_wgrad_rgb DBGS="0 1 2 4" bash tools/anat_c1f.sh 2>&1 | grep -v amdgpu.ids
echo "== ksplit fwd"; timeout -k 10 300 python tools/kbench.py --reps 3 --only conv1_fwd_f32,conv1_fwd_rgb --tune conv1_fwd=4 2>&1 | grep -v amdgpu.ids
