# iCEM: timing per path / rng, and a kernel trace of device-RNG plans
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r43
export TMPDIR=/tmp
timeout -k 10 300 python tools/quick_icem.py > gpurun_out/r43/quick.log 2>&1 || { tail -20 gpurun_out/r43/quick.log; exit 1; }
cat gpurun_out/r43/quick.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r43/kt -o run --output-format csv -- python tools/icem_trace.py device > gpurun_out/r43/kt.log 2>&1 || { tail gpurun_out/r43/kt.log; exit 1; }
python tools/plan_trace.py gpurun_out/r43/kt/run_kernel_trace.csv 1 > gpurun_out/r43/plan.txt || true
cat gpurun_out/r43/plan.txt
