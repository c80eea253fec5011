set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert|skipped" gpurun_out/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench25.json 2> gpurun_out/bench25.err || { tail gpurun_out/bench25.err; exit 1; }
cat gpurun_out/bench25.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof25 -o run --output-format csv -- python bench.py > gpurun_out/prof25.log 2>&1 || { tail gpurun_out/prof25.log; exit 1; }
grep '^{' gpurun_out/prof25.log
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc25_fetch -o run --output-format csv -- tools/mb/mb_linear 8 chainloop 50 > gpurun_out/pmc25_fetch.log 2>&1 || { echo pmc1 failed; tail gpurun_out/pmc25_fetch.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc25_write -o run --output-format csv -- tools/mb/mb_linear 8 chainloop 50 > gpurun_out/pmc25_write.log 2>&1 || { echo pmc2 failed; tail gpurun_out/pmc25_write.log; exit 1; }
echo ALLDONE
