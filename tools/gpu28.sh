set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert|skipped" gpurun_out/pytest_gpu.log | tail -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 tools/mb/mb_linear 8 chain > gpurun_out/mb28.log 2>&1 || { cat gpurun_out/mb28.log; exit 1; }
head -3 gpurun_out/mb28.log
TDMPC_OVERLAP=0 timeout -k 10 120 tools/mb/mb_linear 8 chain > gpurun_out/mb28b.log 2>&1 || { cat gpurun_out/mb28b.log; exit 1; }
head -3 gpurun_out/mb28b.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt28 -o run --output-format csv -- python tools/quick_time.py humanoid-run 8 > gpurun_out/kt28.log 2>&1 || { tail gpurun_out/kt28.log; exit 1; }
grep plan-steps gpurun_out/kt28.log
timeout -k 10 300 python bench.py --steps 30 --no-single --no-replay --no-learner --no-cpu > gpurun_out/bench28.json 2> gpurun_out/bench28.err || { tail -30 gpurun_out/bench28.err; exit 1; }
cat gpurun_out/bench28.json
echo ALLDONE
