# x6 mode 3 with four last-layer items per wave (L512): plan + iCEM parity, L512 timing modes 1 / 3
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r87
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py tests/test_icem.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r87/tests.log 2>&1 || { tail -40 gpurun_out/r87/tests.log; exit 1; }
tail -1 gpurun_out/r87/tests.log
for rep in 1 2; do
for x in 1 3; do
  echo -n "X6=$x "; TDMPC_X6=$x timeout -k 10 120 python tools/quick_time.py humanoid-run-l512 32 2>&1 | grep plan-steps
done; done
