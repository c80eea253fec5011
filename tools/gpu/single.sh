#!/bin/bash
# GPU box: single-env plan() timing by mode, hipBLASLt calibration, plan GPU tests (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 200 python tools/quick_single.py 2>&1 | grep -v amdgpu.ids > $OUT/single.txt || { cat $OUT/single.txt; exit 1; }
cat $OUT/single.txt
timeout -k 10 200 python tools/mm_calibrate.py 2>&1 | grep -v amdgpu.ids > $OUT/mm.txt || { cat $OUT/mm.txt; exit 1; }
cat $OUT/mm.txt
timeout -k 10 900 python -u -m pytest tests/test_dropin_cpu.py tests/test_gpu_plan.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
exit $rc
