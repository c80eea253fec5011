# B = 8 / 16: auto (32-row x6 mode 3) vs 16-row blocks (chain16 x6) vs x6 mode 1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do for B in 8 16; do
  echo -n "auto  "; timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
  echo -n "rb16  "; TDMPC_CHAIN_RB=16 timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
  echo -n "mode1 "; TDMPC_X6=1 timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done
