# x6 mode 3 (4-wave workgroups, 128 columns per wave): parity on the x6 tests, then timing modes 1 / 3
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r83
export TMPDIR=/tmp
TDMPC_X6=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py -x -q -m gpu -k "chain_x6 or building" --timeout 120 --timeout-method thread > gpurun_out/r83/tests.log 2>&1 || { tail -40 gpurun_out/r83/tests.log; exit 1; }
tail -1 gpurun_out/r83/tests.log
for rep in 1 2; do
for B in 32 8; do
for x in 1 3; do
  echo -n "X6=$x "; TDMPC_X6=$x timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done; done
