#!/bin/bash
# GPU box: single-env plan() A/B of the cached pi-row terminal means (TDMPC_PI_CACHE=0 / 1, alternating) (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
for v in 0 1 0 1; do
  TDMPC_PI_CACHE=$v timeout -k 10 200 python tools/quick_single.py > $OUT/single_$v.txt 2>&1 || { tail -20 $OUT/single_$v.txt; exit 1; }
  echo "TDMPC_PI_CACHE=$v"; grep "graft\|graph=True rng=reference/device\|graph=False rng=reference/device" $OUT/single_$v.txt
done
