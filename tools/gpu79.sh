# chain step stamps with phase 0 = input staging only (TDMPC_STAMPS_STAGE), x6, B = 32
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r79
export TMPDIR=/tmp
timeout -k 10 200 tools/mb/mb_linear_st2 32 > gpurun_out/r79/st32.log 2>&1 || { tail -20 gpurun_out/r79/st32.log; exit 1; }
grep -A1 "chain" gpurun_out/r79/st32.log | grep -v blockIdx | grep "avg cycles"
