#!/bin/bash
# Build A/B variants of libppo_hip.so with extra -D flags (container-side):
#   tools/build_variants.sh NAME "-DFOO=1 -DBAR=0" [NAME2 "FLAGS2" ...]
# -> ppo-dash_amd/lib/libppo_hip_NAME.so (csrc/$SRCV.hip — default gemm — recompiled
# with the flags; the other objects of the Makefile's build reused)
set -e
cd "$(dirname "$0")/../ppo-dash_amd"
make -s
V="${SRCV:-gemm}"
XF=""; [ "$V" = gae ] && XF="-ffp-contract=off"
OTHERS=$(ls build/*.o | grep -v -e "^build/$V.o\$" -e '^build/var_')
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -fvisibility=hidden $XF $flags -c csrc/$V.hip -o build/var_$name.o &
done
wait
for o in build/var_*.o; do
  name=${o#build/var_}; name=${name%.o}
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o lib/libppo_hip_$name.so $OTHERS $o
  rm -f $o
done
ls lib/
