set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt24 -o run --output-format csv -- python tools/quick_time.py humanoid-run 8 > gpurun_out/kt24.log 2>&1 || { tail gpurun_out/kt24.log; exit 1; }
grep plan-steps gpurun_out/kt24.log
