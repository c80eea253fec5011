set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r57
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r57/qt -o run --output-format csv -- python tools/quick_time.py humanoid-run 1 > gpurun_out/r57/qt.log 2>&1 || { tail gpurun_out/r57/qt.log; exit 1; }
python tools/plan_trace.py gpurun_out/r57/qt/run_kernel_trace.csv 1 > gpurun_out/r57/plan_b1.txt || true
rm -f gpurun_out/r57/qt/run_kernel_trace.csv
cat gpurun_out/r57/plan_b1.txt
