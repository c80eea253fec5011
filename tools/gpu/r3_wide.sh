#!/bin/bash
# Round 3: the wide step kernel -- parity subset first (stop on any failure), then A/B timing, rocprof, full suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py -v -x --timeout 200 --timeout-method thread \
    -k "wide or bench_shape" > $O/wide_tests.txt 2>&1 || { echo "wide tests failed"; tail -30 $O/wide_tests.txt; exit 1; }
for i in 1 2; do
  for w in 0 1; do
    TDMPC_WIDE=$w timeout -k 10 120 python -u tools/quick_time.py humanoid-run 32 >> $O/ab.txt 2>&1 || exit 1
    echo "  (TDMPC_WIDE=$w)" >> $O/ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u tools/quick_time.py humanoid-run 32 > $O/prof.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo "suite rc=$?" >> $O/gpu_tests.txt
tail -3 $O/gpu_tests.txt
cat $O/ab.txt
