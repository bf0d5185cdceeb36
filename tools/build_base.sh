#!/bin/bash
# Build the library of a git revision (default HEAD) into ppo-dash_amd/lib/libppo_hip_base.so
# for same-box A/B timing (tools/gpu_kb.sh with LIBS="base cur").
set -eu
REV="${1:-HEAD}"
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
W=/tmp/ppo_base_wt
rm -rf "$W"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -f --detach "$W" "$REV" >/dev/null
make -s -C "$W/ppo-dash_amd" -j8 >/dev/null
cp "$W/ppo-dash_amd/lib/libppo_hip.so" "$ROOT/ppo-dash_amd/lib/libppo_hip_base.so"
git -C "$ROOT" worktree remove --force "$W"
echo "built $REV -> ppo-dash_amd/lib/libppo_hip_base.so"
