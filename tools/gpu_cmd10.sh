set -u
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_all.log; [ $rc -eq 0 ] || exit $rc
for o in f32 rgb; do timeout -k 10 600 python bench.py --obs $o --no-cpu-baseline --no-gae-roofline --no-boundary --steps 3 > gpurun_out/bench_obs_$o.log 2>&1 || exit $?; grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus": 1, "steps": 3, "warmup": 1, "ms_per_step": [0-9.]*' gpurun_out/bench_obs_$o.log; done
timeout -k 10 600 python bench.py --force-collectives --no-cpu-baseline --no-gae-roofline --no-boundary --steps 3 > gpurun_out/bench_rccl.log 2>&1 || exit $?; grep -o '"value": [0-9.]*\|"allreduce": {[^}]*}' gpurun_out/bench_rccl.log
