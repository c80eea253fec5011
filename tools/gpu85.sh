# narrow launches: auto row block (16-row f32 chain below half the CUs) vs forced 32-row blocks (x6) at B = 2, 4, 8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
for B in 2 4 8; do
  echo -n "auto "; timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
  echo -n "rb32 "; TDMPC_CHAIN_RB=32 timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done
