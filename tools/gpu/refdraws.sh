#!/bin/bash
# GPU box: one-launch reference-order draws -- parity tests, single-env plan() timing, host profile (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_train_loop.py tests/test_dropin_cpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -k "reference_normals or reference_draws or rng_order or train_loop or golden or dropin or mixed" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 200 python tools/quick_single.py 2>&1 | grep -v amdgpu.ids > $OUT/single.txt || { cat $OUT/single.txt; exit 1; }
cat $OUT/single.txt
timeout -k 10 200 python tools/plan_host_prof.py 2>&1 | grep -v amdgpu.ids > $OUT/host.txt || { cat $OUT/host.txt; exit 1; }
head -1 $OUT/host.txt; tail -2 $OUT/host.txt
