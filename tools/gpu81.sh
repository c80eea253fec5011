# x6 ring without sched barriers around the split (TDMPC_X6_FREE_SCHED build) vs default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
for B in 32 8; do
  echo -n "default "; timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
  echo -n "free    "; TDMPC_LIB_PATH=$GRAFT_REPO_ROOT/tdmpc_amd/libtdmpc_hip_fs.so timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done
