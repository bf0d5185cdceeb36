#!/bin/bash
# same-box end-to-end A/B of library variants (lib/libppo_hip_<name>.so, "cur" = libppo_hip.so),
# each optionally with one environment setting: LIBS="base cur cur@PPO_FUSED_TRUNK=0" ROUNDS=2 ARGS="..." TAG=x
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/${TAG:?}_ab.log
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in ${LIBS:-cur}; do
    v=${spec%%@*}; envset=""; [ "$spec" != "$v" ] && envset=${spec#*@}
    lib=$PWD/ppo-dash_amd/lib/libppo_hip_$v.so; [ $v = cur ] && lib=$PWD/ppo-dash_amd/lib/libppo_hip.so
    echo "== $spec" >> $L
    env $envset PPO_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-gae-roofline --no-boundary ${ARGS:-} > gpurun_out/${TAG}_last.log 2>&1
    rc=$?; grep '^{' gpurun_out/${TAG}_last.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], d['ms_per_step'])" >> $L
    [ $rc -eq 0 ] || { echo "rc=$rc $v"; tail -5 gpurun_out/${TAG}_last.log; exit $rc; }
  done
done
cat $L
