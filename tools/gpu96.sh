# x6 mode-3 weight ring depth 3 (X6_D=3 build: step kernel at 256 VGPRs, pi / Q with a few spills) vs 2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do for B in 32 8; do
  echo -n "D2 "; timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
  echo -n "D3 "; TDMPC_LIB_PATH=$GRAFT_REPO_ROOT/tdmpc_amd/libtdmpc_hip_d3.so timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done
