#!/bin/bash
# Round 4 GPU check: selected pytest targets (args after OUT) then the default bench line.
#   tools/gpu/r4_quick.sh OUT [pytest targets...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 \
    || { tail -40 $OUT/tests.log; exit 1; }
  grep -E "passed|failed" $OUT/tests.log | tail -2
fi
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
