#!/bin/bash
# persistent BPTT: parity + fail-safe tests, then the c5 bench (persistent vs step launches)
set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_failsafe.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gru or failsafe or timeout or action" > gpurun_out/t19.log 2>&1; rc=$?; tail -3 gpurun_out/t19.log; [ $rc -eq 0 ] || exit $rc
for p in 1 0; do echo "== c5 gru-persist $p"; timeout -k 10 400 python bench.py --recurrent --gru-persist $p --no-cpu-baseline --no-gae-roofline --no-boundary > gpurun_out/b19_$p.log 2>&1 || { tail -5 gpurun_out/b19_$p.log; exit 1; }; grep '^{' gpurun_out/b19_$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernel_rooflines',{}); print(d['value'], d['ms_per_step'], {n: k[n].get('ms_per_iteration') for n in k if 'gru' in n})"; done
