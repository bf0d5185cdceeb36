#!/bin/bash
# Same-box A/B of the c3 bench line under two environment settings, alternating:
#   A_ENV="PPO_PERM_PREFETCH=0" B_ENV="PPO_PERM_PREFETCH=1" ROUNDS=2 bash tools/ab_env.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
for r in $(seq ${ROUNDS:-2}); do
  for E in "${A_ENV:?}" "${B_ENV:?}"; do
    echo "--- $E"
    env $E timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-gae-roofline --no-boundary ${ARGS:-} 2>&1 \
      | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
