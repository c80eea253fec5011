#!/bin/bash
# A/B of an environment knob on humanoid B=32 (alternating, same box): r3_envab.sh VAR v1 v2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
var=$1; shift
for i in 1 2 3; do
  for v in "$@"; do
    env "$var=$v" timeout -k 10 120 python -u tools/quick_time.py humanoid-run 32 2>&1 | grep -v amdgpu.ids | sed "s/^/$var=$v: /" || exit 1
  done
done
