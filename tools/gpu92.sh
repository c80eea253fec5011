# x6 pipelined split (X6_PIPE=1, default build) vs not (X6_PIPE=0 build): parity (x6 paths), timing B = 32, 8
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r92
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py -x -q -m gpu -k "x6 or chain]" --timeout 200 --timeout-method thread > gpurun_out/r92/tests.log 2>&1 || { tail -40 gpurun_out/r92/tests.log; exit 1; }
tail -1 gpurun_out/r92/tests.log
for rep in 1 2; do
for B in 32 8; do
  echo -n "pipe   "; timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
  echo -n "nopipe "; TDMPC_LIB_PATH=$GRAFT_REPO_ROOT/tdmpc_amd/libtdmpc_hip_nopipe.so timeout -k 10 120 python tools/quick_time.py humanoid-run $B 2>&1 | grep plan-steps
done; done
