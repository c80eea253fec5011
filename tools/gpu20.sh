set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { tail gpurun_out/bench20.err; exit 1; }
cat gpurun_out/bench20.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof20 -o run --output-format csv -- python bench.py > gpurun_out/prof20.log 2>&1 || { tail gpurun_out/prof20.log; exit 1; }
grep '^{' gpurun_out/prof20.log
echo ALLDONE
