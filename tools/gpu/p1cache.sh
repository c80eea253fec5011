#!/bin/bash
# GPU box: plan parity tests (persist path included) with plan1's cached pi-row terminal means, then the
# single-env timings (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python tools/quick_single.py > $OUT/single.txt 2>&1 || { tail -20 $OUT/single.txt; exit 1; }
grep -v amdgpu.ids $OUT/single.txt
