# x6 chain kernels: parity on every GPU plan test with path chain_x6, then A/B timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r72
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py -x -q -m gpu -k "x6" --timeout 120 --timeout-method thread > gpurun_out/r72/tests.log 2>&1; rc=$?
tail -30 gpurun_out/r72/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for B in 32 8; do
for x in 0 1; do
  echo -n "X6=$x "; TDMPC_X6=$x timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done
