#!/bin/bash
# Kernel iteration loop on one box: a parity subset (stop on failure), then an A/B of an environment knob on a config's
# batch plan (alternating runs of tools/quick_time.py), then a rocprofv3 kernel trace of the default side.
#   tools/gpu/iter.sh OUT "PYTEST -k EXPR" VAR "v1 v2" [config] [envs]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1; K=$2; VAR=$3; VALS=$4; CFG=${5:-humanoid-run}; B=${6:-32}
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_configs.py tests/test_gpu_sharded.py -m gpu -v -x \
      --timeout 200 --timeout-method thread -k "$K" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
  grep -E "passed|failed" $O/tests.txt | tail -1
fi
for i in 1 2 3; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 120 python -u tools/quick_time.py $CFG $B 2>&1 | grep -v amdgpu.ids | sed "s/^/$VAR=$v: /" || exit 1
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u tools/quick_time.py $CFG $B > $O/prof.log 2>&1 || exit 1
python tools/rocpd_summary.py $O/prof/run_results.db 12 --grid > $O/prof_summary.txt 2>&1
cut -c1-150 $O/prof_summary.txt | head -16
