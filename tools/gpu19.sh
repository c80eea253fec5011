set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt19 -o run --output-format csv -- python tools/quick_time.py humanoid-run 1 > gpurun_out/kt19.log 2>&1 || { tail gpurun_out/kt19.log; exit 1; }
tail -1 gpurun_out/kt19.log
