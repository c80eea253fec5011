set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert|skipped" gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 tools/mb/mb_linear_st 8 > gpurun_out/mb23_st.log 2>&1 || { cat gpurun_out/mb23_st.log; exit 1; }
grep -v "blockIdx" gpurun_out/mb23_st.log | grep -v "S2 "
timeout -k 10 300 python tools/quick_time.py humanoid-run 8
echo ALLDONE
