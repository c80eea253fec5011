# x6 split kernels (single env): parity on the split_x6 path, then timing of one env and B = 2, 4 (auto path)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r77
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py -x -q -m gpu -k "split_x6" --timeout 120 --timeout-method thread > gpurun_out/r77/tests.log 2>&1 || { tail -40 gpurun_out/r77/tests.log; exit 1; }
tail -1 gpurun_out/r77/tests.log
for rep in 1 2; do
for B in 1 2; do
for x in 0 1; do
  echo -n "X6=$x "; TDMPC_X6=$x timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done; done
