# x6 chain16 (layers 1-2 on the bf16 MFMA for 16-row blocks): plan + iCEM parity incl. path "chain", timing B = 1, 2, 4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r90
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py tests/test_icem.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r90/tests.log 2>&1 || { tail -40 gpurun_out/r90/tests.log; exit 1; }
tail -1 gpurun_out/r90/tests.log
for rep in 1 2; do
for B in 1 2 4; do
for x in 0 3; do
  echo -n "X6=$x "; TDMPC_X6=$x timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done; done
