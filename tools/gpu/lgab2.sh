#!/bin/bash
# GPU box: learner update time A/B over an env knob, interleaved (args: OUT VAR v1 v2 [reps])
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; VAR=$2; V1=$3; V2=$4; N=${5:-3}; mkdir -p $OUT
for i in $(seq $N); do
  for v in $V1 $V2; do
    echo -n "$VAR=$v " >> $OUT/ab.txt
    env $VAR=$v REPS=40 timeout -k 10 200 python tools/quick_learner.py 2>&1 | grep -v amdgpu.ids | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['graph']['ms_per_update'])" >> $OUT/ab.txt || { cat $OUT/ab.txt; exit 1; }
  done
done
cat $OUT/ab.txt
