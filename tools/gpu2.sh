set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -20
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof1 -o run --output-format csv -- python tools/quick_time.py humanoid-run 1 > gpurun_out/prof1.log 2>&1; echo "prof rc=$?"
tail -3 gpurun_out/prof1.log
find gpurun_out/prof1 -name "*stats*" | head
