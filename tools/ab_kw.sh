cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do for t in 8 9; do
  echo "--- conv1_wgrad=$t"
  timeout -k 10 300 python bench.py --tune conv1_wgrad=$t > gpurun_out/ab_kw_${t}_${r}.json 2> gpurun_out/ab_kw_err.log || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_kw_${t}_${r}.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
done; done
