# per-phase cycles of the chain step workgroups (s_memtime stamps), x6 vs f32, B = 32
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r78
export TMPDIR=/tmp
for x in 1 0; do
  TDMPC_X6=$x timeout -k 10 200 tools/mb/mb_linear_st 32 > gpurun_out/r78/st32_x$x.log 2>&1 || { tail -20 gpurun_out/r78/st32_x$x.log; exit 1; }
  echo "X6=$x"; grep -A1 "chain" gpurun_out/r78/st32_x$x.log | grep -v blockIdx
done
