# wave-parallel CEM refit: full GPU suite, one-env timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r94
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r94/tests.log 2>&1 || { tail -40 gpurun_out/r94/tests.log; exit 1; }
tail -1 gpurun_out/r94/tests.log
for rep in 1 2; do for B in 1 32; do timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps; done; done
