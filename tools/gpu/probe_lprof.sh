#!/bin/bash
# GPU box: x6 stream probe + a rocprofv3 kernel trace of the learner leg (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 120 tools/mb/x6_stream > $OUT/probe.txt 2>&1 || { cat $OUT/probe.txt; exit 1; }
cat $OUT/probe.txt
REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lp -o run -- python3 tools/quick_learner.py > $OUT/lp.log 2>&1 || { tail -20 $OUT/lp.log; exit 1; }
tail -2 $OUT/lp.log
python3 tools/learner_prof.py $(find $OUT/lp -name '*kernel_trace.csv' | head -1) 10 > $OUT/learner_kernels.txt
cat $OUT/learner_kernels.txt
