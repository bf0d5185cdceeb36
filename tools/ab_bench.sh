#!/bin/bash
# same-box end-to-end A/B of library variants: LIBS="base cur wt" ROUNDS=2 ARGS="..." TAG=x
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/${TAG:?}_ab.log
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-cur}; do
    lib=$PWD/ppo-dash_amd/lib/libppo_hip_$v.so; [ $v = cur ] && lib=$PWD/ppo-dash_amd/lib/libppo_hip.so
    echo "== $v" >> $L
    PPO_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-gae-roofline --no-boundary ${ARGS:-} > gpurun_out/${TAG}_last.log 2>&1
    rc=$?; grep '^{' gpurun_out/${TAG}_last.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" >> $L
    [ $rc -eq 0 ] || { echo "rc=$rc $v"; tail -5 gpurun_out/${TAG}_last.log; exit $rc; }
  done
done
cat $L
