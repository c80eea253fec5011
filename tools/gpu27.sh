set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert|skipped" gpurun_out/pytest_gpu.log | tail -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 20 --no-single > gpurun_out/bench27.json 2> gpurun_out/bench27.err || { tail -30 gpurun_out/bench27.err; exit 1; }
cat gpurun_out/bench27.json
echo ALLDONE
