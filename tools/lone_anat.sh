#!/bin/bash
# conv2 lone-pixel kernel anatomy (timing only): rocprofv3 kernel stats of kbench
# conv2_fwd_mask per library variant (tools/build_variants.sh: nosplit, nostore, nomma)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
for L in cur ${LIBS:-nosplit nostore nomma}; do
  lib=$PWD/ppo-dash_amd/lib/libppo_hip_$L.so; [ $L = cur ] && lib=$PWD/ppo-dash_amd/lib/libppo_hip.so
  PPO_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/an_$L -o kb -- python3 tools/kbench.py --reps 5 --z1 256 --z2 256 --only ${KB:-conv2_fwd_mask} > /dev/null 2>&1 || exit 1
  echo "== $L"; grep -h "lone" gpurun_out/an_$L/kb_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-40,90-200
done
