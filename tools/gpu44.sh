# iCEM fused device RNG: GPU tests + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r44
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r44/tests.log 2>&1 || { tail -40 gpurun_out/r44/tests.log; exit 1; }
tail -2 gpurun_out/r44/tests.log
timeout -k 10 300 python tools/quick_icem.py > gpurun_out/r44/quick.log 2>&1 || { tail -20 gpurun_out/r44/quick.log; exit 1; }
cat gpurun_out/r44/quick.log
