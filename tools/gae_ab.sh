#!/bin/bash
# GAE roofline (bench.py's gae_roofline leg, 1M lanes x 128) per library variant:
#   LIBS="cur u16" bash tools/gae_ab.sh   (variants: tools/build_variants.sh with SRCV=gae)
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
for L in ${LIBS:-cur}; do
  if [ "$L" = cur ]; then unset PPO_HIP_LIB; else export PPO_HIP_LIB=$PWD/ppo-dash_amd/lib/libppo_hip_$L.so; fi
  echo "--- $L"
  timeout -k 10 120 python -c "
import sys, torch; sys.path[:0] = ['.', 'ppo-dash_amd']
import bench
r = bench.gae_roofline(torch.device('cuda'), 1 << 20)
print({k: r[k] for k in ('achieved', 'frac', 'ms_per_launch')})" 2>&1 | grep -v amdgpu.ids
  rc=$?; [ $rc -eq 0 ] || exit $rc
done
