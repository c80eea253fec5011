#!/bin/bash
# GPU box: learner update time A/B of two library builds, interleaved (args: OUT libA libB [reps])
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; LA=$2; LB=$3; N=${4:-3}; mkdir -p $OUT
for i in $(seq $N); do
  for L in $LA $LB; do
    echo -n "$L " >> $OUT/ab.txt
    TDMPC_LIB_PATH=$PWD/tdmpc_amd/$L REPS=40 timeout -k 10 200 python tools/quick_learner.py 2>&1 | grep -v amdgpu.ids | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['graph']['ms_per_update'])" >> $OUT/ab.txt || { cat $OUT/ab.txt; exit 1; }
  done
done
cat $OUT/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_learner.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
exit $rc
