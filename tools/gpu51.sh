set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r51
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r51/tests.log 2>&1 || { tail -40 gpurun_out/r51/tests.log; exit 1; }
tail -1 gpurun_out/r51/tests.log
for b in 1 8 32; do timeout -k 10 300 python tools/quick_time.py quadruped-run-pixels $b 2>&1 | grep plan-steps; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r51/qt -o run --output-format csv -- python tools/quick_time.py quadruped-run-pixels 32 > gpurun_out/r51/qt.log 2>&1 || { tail gpurun_out/r51/qt.log; exit 1; }
grep -E "conv|Name" gpurun_out/r51/qt/run_kernel_stats.csv | cut -c1-160
rm -f gpurun_out/r51/qt/run_kernel_trace.csv
