#!/bin/bash
# Per-step shader stamps of the wide step kernels (the -DWS_STAMPS variant library), both kernel versions, then an A/B
# of the plan time (tools/gpu/stamps.sh [OUT])
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-st}; mkdir -p $O
for v in 1 0; do
  TDMPC_WIDE2=$v TDMPC_LIB_PATH=$PWD/tdmpc_amd/libtdmpc_hip_ws.so timeout -k 10 200 python -u tools/ws_stamps.py 32 > $O/stamps_v$v.txt 2>&1 || exit 1
  grep -v amdgpu.ids $O/stamps_v$v.txt | head -5
done
for i in 1 2; do
  for v in 0 1; do
    TDMPC_WIDE2=$v timeout -k 10 120 python -u tools/quick_time.py humanoid-run 32 2>&1 | grep -v amdgpu.ids | sed "s/^/WIDE2=$v: /" || exit 1
  done
done
