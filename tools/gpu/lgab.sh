#!/bin/bash
# GPU box: lg_gemm bench + learner update time for library variants (args: OUT lib...)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for L in "$@"; do
  echo "== $L" >> $OUT/ab.txt
  TDMPC_LIB_PATH=$PWD/tdmpc_amd/$L timeout -k 10 200 python tools/lg_gemm_bench.py 2>&1 | grep -v amdgpu.ids | grep -v "rel err 1.0e+00" >> $OUT/ab.txt || exit 1
  TDMPC_LIB_PATH=$PWD/tdmpc_amd/$L REPS=30 timeout -k 10 200 python tools/quick_learner.py 2>&1 | grep -v amdgpu.ids | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('learner', d['graph'])" >> $OUT/ab.txt || exit 1
done
cat $OUT/ab.txt
