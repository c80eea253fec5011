# split-step kernel: parity (forced path 'split'), then single-env timing with it on / off
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r58
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r58/tests.log 2>&1 || { tail -40 gpurun_out/r58/tests.log; exit 1; }
tail -1 gpurun_out/r58/tests.log
for sp in 1 0; do for b in 1 2 4; do echo "split=$sp $(TDMPC_SPLIT=$sp timeout -k 10 120 python tools/quick_time.py humanoid-run $b 2>&1 | grep plan-steps)"; done; done
TDMPC_SPLIT=1 timeout -k 10 300 python tools/quick_icem.py 2>&1 | grep "path=auto"
