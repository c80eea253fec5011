# kernel trace of one-env plans (graph replay): per-kernel breakdown of one plan
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r89
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r89/kt -o run --output-format csv -- python tools/quick_time.py humanoid-run 1 > gpurun_out/r89/kt.log 2>&1 || { tail gpurun_out/r89/kt.log; exit 1; }
python tools/plan_trace.py gpurun_out/r89/kt/run_kernel_trace.csv 1 > gpurun_out/r89/plan_b1.txt
rm -f gpurun_out/r89/kt/run_kernel_trace.csv
cat gpurun_out/r89/plan_b1.txt | head -40
