#!/bin/bash
# GPU box: lg_gemm bench + learner time with the x6 products on / off, learner tests with x6 (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
for v in 0 1; do
  echo "== TDMPC_LG_X6=$v" >> $OUT/ab.txt
  TDMPC_LG_X6=$v timeout -k 10 200 python tools/lg_gemm_bench.py 2>&1 | grep -v amdgpu.ids | grep "k   512\|k  2560\|k   121" >> $OUT/ab.txt || { cat $OUT/ab.txt; exit 1; }
done
for i in 1 2; do for v in 0 1; do
  echo -n "learner TDMPC_LG_X6=$v " >> $OUT/ab.txt
  TDMPC_LG_X6=$v REPS=40 timeout -k 10 200 python tools/quick_learner.py 2>&1 | grep -v amdgpu.ids | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['graph']['ms_per_update'])" >> $OUT/ab.txt || { cat $OUT/ab.txt; exit 1; }
done; done
cat $OUT/ab.txt
TDMPC_LG_X6=1 timeout -k 10 600 python -u -m pytest tests/test_learner.py tests/test_gpu_train_loop.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -25 $OUT/tests.log
exit $rc
