#!/bin/bash
# GPU box check: parity suite, smoke, default bench (and optionally a rocprof kernel-trace of the bench).
#   tools/gpu/suite.sh OUT [tests] [smoke] [bench] [prof]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for stage in "$@"; do
  case $stage in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
             > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }; tail -3 $OUT/tests.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1 ;;
    bench) timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
           cat $OUT/bench.json ;;
    prof)  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-single --no-replay --no-learner --no-icem --no-exact \
             > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; } ;;
  esac
done
