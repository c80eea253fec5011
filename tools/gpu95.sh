# A/B: wave-parallel CEM refit (default build) vs the sequential one (previous commit's kernels), one env and B = 32
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2 3; do for B in 1 8; do
  echo -n "new "; timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
  echo -n "old "; TDMPC_LIB_PATH=$GRAFT_REPO_ROOT/tdmpc_amd/libtdmpc_hip_old.so timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done
