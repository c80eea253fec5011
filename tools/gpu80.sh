# x6 L2 warm-up: parity (x6 paths), stamps, timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r80
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py -x -q -m gpu -k "x6" --timeout 120 --timeout-method thread > gpurun_out/r80/tests.log 2>&1 || { tail -40 gpurun_out/r80/tests.log; exit 1; }
tail -1 gpurun_out/r80/tests.log
timeout -k 10 200 tools/mb/mb_linear_st2 32 > gpurun_out/r80/st32.log 2>&1 || { tail -20 gpurun_out/r80/st32.log; exit 1; }
grep -A1 "chain" gpurun_out/r80/st32.log | grep -v blockIdx | grep "avg cycles"
grep "step_next N rows (chain)\|policy T rows (chain)\|terminal_q T rows (chain)" gpurun_out/r80/st32.log
for B in 32 8; do
  timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done
