set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_half.py -m gpu -x -q --timeout 300 --timeout-method thread -k "conv1_wgrad or half" > gpurun_out/t11.log 2>&1; rc=$?; tail -3 gpurun_out/t11.log; [ $rc -eq 0 ] || exit $rc
for t in 5 6; do echo "== conv1_wgrad tune $t"; timeout -k 10 300 python tools/kbench.py --reps 5 --only conv1_wgrad --tune conv1_wgrad=$t 2>&1 | grep -v amdgpu; done
echo "== tune 6 anatomy"; for d in 1 2 4; do timeout -k 10 300 python tools/kbench.py --reps 5 --only conv1_wgrad --tune conv1_wgrad=6,stagger=$((16*d+2)) 2>&1 | grep conv1_wgrad; done
