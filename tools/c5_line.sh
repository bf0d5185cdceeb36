cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-gae-roofline --no-boundary --recurrent --num-steps 256 > gpurun_out/r05_zc_c5.log 2>&1 || exit 1
grep '^{' gpurun_out/r05_zc_c5.log | tail -1 > gpurun_out/r05_zc_c5.json
python -c "import json; d=json.load(open('gpurun_out/r05_zc_c5.json')); print('c5', d['value'], d['ms_per_step'])"
