set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t33.log 2>&1 || { tail -30 gpurun_out/t33.log; exit 1; }
tail -3 gpurun_out/t33.log
timeout -k 10 300 python tools/quick_icem.py > gpurun_out/q33.log 2>&1 || { tail gpurun_out/q33.log; exit 1; }
cat gpurun_out/q33.log
