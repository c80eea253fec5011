set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 tools/mb/mb_linear 8 > gpurun_out/mb12.log 2>&1 || exit 1; sed -n 1,8p gpurun_out/mb12.log
timeout -k 10 200 tools/mb/mb_linear 8 sweep > gpurun_out/sweep8.log 2>&1 || exit 1; cat gpurun_out/sweep8.log
timeout -k 10 200 tools/mb/mb_linear 1 sweep > gpurun_out/sweep1.log 2>&1 || exit 1; cat gpurun_out/sweep1.log
echo ALLDONE
