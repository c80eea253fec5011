set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/mb/mb_linear_st 8 > gpurun_out/mb22_st.log 2>&1 || { cat gpurun_out/mb22_st.log; exit 1; }
grep -v "blockIdx" gpurun_out/mb22_st.log
