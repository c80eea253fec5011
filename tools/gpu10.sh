set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit 1
for v in 0 1; do echo "lds variant $v"; TDMPC_LDS_VARIANT=$v timeout -k 10 120 tools/mb/mb_linear 8 | head -6 || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace -T -d gpurun_out/kt10 -o run --output-format csv -- python tools/quick_time.py humanoid-run 8 > gpurun_out/kt10.log 2>&1; echo "kt rc=$?"
