set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r47
export TMPDIR=/tmp
timeout -k 10 200 tools/mb/mb_linear_st 32 > gpurun_out/r47/st32.log 2>&1 || { tail -20 gpurun_out/r47/st32.log; exit 1; }
grep -A2 "chain" gpurun_out/r47/st32.log
timeout -k 10 200 tools/mb/mb_linear_st 8 > gpurun_out/r47/st8.log 2>&1 || { tail -20 gpurun_out/r47/st8.log; exit 1; }
grep -A2 "chain" gpurun_out/r47/st8.log
