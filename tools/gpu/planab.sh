#!/bin/bash
# GPU box: plan_batch time A/B of two library builds, interleaved (args: OUT libA libB "config B ..." [reps])
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; LA=$2; LB=$3; CASES=$4; N=${5:-2}; mkdir -p $OUT
for i in $(seq $N); do
  for L in $LA $LB; do
    set -- $CASES
    while [ $# -ge 2 ]; do
      echo -n "$L " >> $OUT/ab.txt
      TDMPC_LIB_PATH=$PWD/tdmpc_amd/$L timeout -k 10 200 python tools/quick_time.py $1 $2 2>&1 | grep plan-steps >> $OUT/ab.txt || { cat $OUT/ab.txt; exit 1; }
      shift 2
    done
  done
done
cat $OUT/ab.txt
