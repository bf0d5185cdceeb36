set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -q -x --timeout 120 --timeout-method thread -k "gru or recurrent" > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
for L in 0 1; do
  timeout -k 10 400 python bench.py --gru-persist $L --recurrent --num-steps 256 --no-cpu-baseline --no-gae-roofline --no-boundary --steps 2 --warmup 1 > gpurun_out/c5_$L.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/c5_$L.log') if l.startswith('{')][-1])
print('$L', d['value'], {k: d['kernel_rooflines'][k]['avg_launch_ms'] for k in ('gru_seq_fwd','gru_seq_bwd')})"
done
