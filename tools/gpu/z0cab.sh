#!/bin/bash
# GPU box: plan parity tests with the per-env z0 first-layer split at t = 0, then a bench A/B (TDMPC_Z0C=0 / 1) (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
SHORT="--steps 30 --warmup 3 --no-cpu --no-single --no-replay --no-learner --no-icem --no-exact --no-roofline --sweep= --also="
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in 0 1 0 1; do
  TDMPC_Z0C=$v timeout -k 10 300 python bench.py $SHORT > $OUT/b$v.json 2> $OUT/b$v.err || { tail -20 $OUT/b$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$v.json')); print('Z0C=$v', d['value'], d['ms_per_step'])"
done
