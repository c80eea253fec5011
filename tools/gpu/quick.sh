#!/bin/bash
# GPU box: quick_time for a few batch sizes (args: OUT config B...)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; CFG=$2; shift 2
mkdir -p $OUT
for B in "$@"; do
  timeout -k 10 120 python tools/quick_time.py $CFG $B >> $OUT/quick.log 2>&1 || exit 1
done
cat $OUT/quick.log
