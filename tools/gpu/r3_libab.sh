#!/bin/bash
# A/B of in-tree library variants (tdmpc_amd/libtdmpc_hip_<v>.so) on humanoid B=32, alternating, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TDMPC_WIDE=${TDMPC_WIDE:-1}
for i in 1 2 3; do
  for v in "$@"; do
    TDMPC_LIB_PATH=$PWD/tdmpc_amd/libtdmpc_hip_$v.so timeout -k 10 120 python -u tools/quick_time.py humanoid-run 32 2>&1 | grep -v amdgpu.ids | sed "s/^/$v: /" || exit 1
  done
done
