# x6 chain last-layer ring depth: X6_D3 = 2 (default build) vs 4 vs 6
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
for B in 32 8; do
  echo -n "D3=2 "; timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
  for d in 4 6; do
    echo -n "D3=$d "; TDMPC_LIB_PATH=$GRAFT_REPO_ROOT/tdmpc_amd/libtdmpc_hip_d$d.so timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
  done
done; done
