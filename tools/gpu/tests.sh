#!/bin/bash
# GPU box: run selected pytest targets (args) under a time limit; log to gpurun_out/$OUT/tests.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest "$@" -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -40 $OUT/tests.log
exit $rc
