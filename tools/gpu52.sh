# single-env / small-batch: per-head chain thresholds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r52
export TMPDIR=/tmp
for q in 64 32 16; do for p in 64 16; do for st in 64 32; do
  for b in 1 2; do
    echo "Q=$q PI=$p STEP=$st $(TDMPC_CHAIN_WGS_Q=$q TDMPC_CHAIN_WGS_PI=$p TDMPC_CHAIN_WGS_STEP=$st timeout -k 10 120 python tools/quick_time.py humanoid-run $b 2>&1 | grep plan-steps)"
  done
done; done; done
