#!/bin/bash
# GPU box: learner update time, learner GPU tests, a kernel trace of the learner leg (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift; mkdir -p $OUT
REPS=30 timeout -k 10 200 python tools/quick_learner.py 2>&1 | grep -v amdgpu.ids | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('learner', d['graph'], d['eager'])" >> $OUT/ab.txt || { cat $OUT/ab.txt; exit 1; }

cat $OUT/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_learner.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lp -o run -- python3 tools/quick_learner.py > $OUT/lp.log 2>&1 || { tail -20 $OUT/lp.log; exit 1; }
python3 tools/learner_prof.py $(find $OUT/lp -name '*kernel_trace.csv' | head -1) 10 > $OUT/learner_kernels.txt
head -12 $OUT/learner_kernels.txt
