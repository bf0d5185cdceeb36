#!/bin/bash
# Round-6 GPU call driver: the named steps in order, each under its own time limit,
# stopping at the first failure (no GPU step after a fault, abort or timeout).
#   TAG=r06_x STEPS="tests gru kbench bench" K="-k trunk" bash tools/r06.sh
# tests: pytest -m gpu (K selects), smoke: __graft_entry__.smoke(), gru: whole-sequence GRU
# timings (step launches vs persistent), kbench: per-kernel timings at the c3 minibatch, bench: the c3 line (BENCH_ARGS),
# c5: the recurrent line.  Logs: gpurun_out/<TAG>_<step>.log
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
TAG="${TAG:?set TAG}"
mkdir -p gpurun_out
run() {   # name seconds cmd...
  local name=$1 secs=$2; shift 2
  local log=gpurun_out/${TAG}_${name}.log
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "$log" | tail -${TAILN:-6}
  if [ $rc -ne 0 ]; then echo "== $name rc=$rc"; grep -E "FAILED|Error|error" "$log" | head -20; exit $rc; fi
}
for st in ${STEPS:-tests}; do
  case $st in
    tests) run tests ${TESTS_S:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${KEXPR:+-k "$KEXPR"} ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    gru) run gru 240 python -u tools/gru_bench.py --modes 0,3 ;;
    kbench) run kbench 240 python -u tools/kbench.py ${KB_ARGS:-} ;;
    bench) run bench 500 python -u bench.py ${BENCH_ARGS:-} ;;
    kbab) run kbab 600 bash -c 'for r in 1 2; do for L in ${KB_LIBS:-base cur}; do echo "--- lib=$L"; if [ $L = cur ]; then unset PPO_HIP_LIB; else export PPO_HIP_LIB=ppo-dash_amd/lib/libppo_hip_$L.so; fi; timeout -k 10 150 python tools/kbench.py --reps 10 ${KB_ARGS:-} || exit 1; done; done' ;;
    ab) TAILN=12 run abrun 900 env TAG=${TAG} LIBS="${AB_LIBS:-base cur}" ROUNDS=${AB_ROUNDS:-2} ARGS="${AB_ARGS:-}" bash tools/ab_bench.sh ;;
    kbtune) run kbtune 600 bash -c 'for r in 1 2; do for T in ${KB_TUNES:?}; do echo "--- tune=$T"; timeout -k 10 150 python tools/kbench.py --reps 10 --tune $T ${KBT_ARGS:-} || exit 1; done; done' ;;
    sqab) run sqab 900 bash -c 'for L in ${SQ_LIBS:-base cur}; do if [ $L = cur ]; then unset PPO_HIP_LIB; else export PPO_HIP_LIB=$PWD/ppo-dash_amd/lib/libppo_hip_$L.so; fi; ONLY=${SQ_ONLY:?} bash tools/pmc_sq.sh || exit 1; rm -rf gpurun_out/pmc1_$L; mv gpurun_out/pmc1 gpurun_out/pmc1_$L; done' ;;
    c5) run c5 600 python -u bench.py --recurrent --num-steps 256 --no-cpu-baseline --no-gae-roofline --no-boundary ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "== all done"
