set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 tools/mb/mb_linear 8 chaind > gpurun_out/mb31.log 2>&1 || { cat gpurun_out/mb31.log; exit 1; }
cat gpurun_out/mb31.log
