set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt32 -o run --output-format csv -- python tools/quick_icem.py > gpurun_out/kt32.log 2>&1 || { tail gpurun_out/kt32.log; exit 1; }
grep "ms/call" gpurun_out/kt32.log
python tools/prof_summary.py gpurun_out/kt32/run_kernel_trace.csv 43 > gpurun_out/kt32_summary.txt
head -25 gpurun_out/kt32_summary.txt
rm -f gpurun_out/kt32/run_kernel_trace.csv
