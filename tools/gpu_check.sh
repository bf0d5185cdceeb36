#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof.  Every GPU step has
# its own time limit; a fault/abort/timeout (rc not 0/1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="${STEPS:-pytest smoke bench}"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!! stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
export PYTHONDONTWRITEBYTECODE=1
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    pytestall) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    new) run pytest_new 1100 python -u -m pytest ${TESTS:-tests/test_failsafe.py tests/test_rccl.py tests/test_evaluation.py} ${KSEL:+-k "$KSEL"} -m gpu -x -v -s --timeout 600 --timeout-method thread ;;
    obsbench) for o in f32 rgb; do run bench_obs_$o 900 python bench.py --obs $o --no-cpu-baseline --no-gae-roofline --no-boundary --steps 3; done ;;
    rcclbench) run bench_rccl 900 python bench.py --force-collectives --no-cpu-baseline --no-gae-roofline --no-boundary --steps 3 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    benchq) run bench 900 python bench.py --no-cpu-baseline --steps 2 --warmup 1 ;;
    half) run pytest_half 600 python -u -m pytest tests/test_half.py -m gpu -v --timeout 300 --timeout-method thread ;;
    c5bench) run bench_c5 900 python bench.py --recurrent --num-steps 256 --no-cpu-baseline --no-gae-roofline --no-boundary ;;
    halfbench) run bench_half 900 python bench.py --half-precision --no-cpu-baseline --no-gae-roofline --no-boundary ;;
    c5prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          run rocprof_c5 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --recurrent --num-steps 256 --no-cpu-baseline --no-gae-roofline --no-boundary --steps 2 --warmup 1 ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          run rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-gae-roofline --steps 2 --warmup 1 ;;
  esac
done
echo "== all done"
