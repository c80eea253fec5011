#!/bin/bash
# Learner check on one box: the learner / train-loop / adam parity tests, then an A/B of an environment knob on the
# humanoid update time (tools/quick_learner.py), alternating.   tools/gpu/learner_ab.sh OUT VAR "v1 v2"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; VAR=$2; VALS=$3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_learner.py tests/test_gpu_train_loop.py tests/test_gpu_adam.py -m gpu -v -x \
    --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
grep -E "passed|failed" $O/tests.txt | tail -1
for i in 1 2 3; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 120 python -u tools/quick_learner.py humanoid-run 2>&1 | grep -v amdgpu.ids | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$VAR=$v', d['graph'])" || exit 1
  done
done
