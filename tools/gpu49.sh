set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r49
export TMPDIR=/tmp
timeout -k 10 300 python tools/quick_single.py > gpurun_out/r49/single.log 2>&1 || { tail -20 gpurun_out/r49/single.log; exit 1; }
cat gpurun_out/r49/single.log
