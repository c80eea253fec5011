#!/bin/bash
# GPU box: one-launch reference-order draws -- parity tests, then single-env plan() timing (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -k "reference_normals or reference_draws or rng_order" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -12 $OUT/tests.log
timeout -k 10 200 python tools/quick_single.py 2>&1 | grep -v amdgpu.ids > $OUT/single.txt || { cat $OUT/single.txt; exit 1; }
cat $OUT/single.txt
