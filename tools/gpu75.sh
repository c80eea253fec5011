# x6 planes mode (TDMPC_X6=2): parity of the x6 path tests, then timing modes 1 / 2 / off
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r75
export TMPDIR=/tmp
TDMPC_X6=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py -x -q -m gpu -k "x6" --timeout 120 --timeout-method thread > gpurun_out/r75/tests.log 2>&1 || { tail -30 gpurun_out/r75/tests.log; exit 1; }
tail -1 gpurun_out/r75/tests.log
for rep in 1 2; do
for B in 32 8; do
for x in 0 1 2; do
  echo -n "X6=$x "; TDMPC_X6=$x timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done; done
