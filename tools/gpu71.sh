set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
for B in 32 8; do
for dd in 4 6; do
  echo -n "D=$dd "; TDMPC_CHAIN_D=$dd timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done; done
