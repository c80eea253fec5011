set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/bench30.json 2> gpurun_out/bench30.err || { tail -30 gpurun_out/bench30.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof30 -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/prof30.log 2>&1 || { tail gpurun_out/prof30.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof30/run_kernel_trace.csv > gpurun_out/prof30_summary.txt
python tools/plan_trace.py gpurun_out/prof30/run_kernel_trace.csv 1 > gpurun_out/prof30_plan_b1.txt || true
rm -f gpurun_out/prof30/run_kernel_trace.csv
du -sh gpurun_out
echo ALLDONE
