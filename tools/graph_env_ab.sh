#!/bin/bash
# The humanoid learner update time (graph replay, tools/quick_learner.py) under HIP runtime graph settings, alternated
# 3 rounds: each argument is one setting ("base" = none, or VAR=value[,VAR=value]).   bash tools/graph_env_ab.sh OUT SET...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for i in 1 2 3; do
  for s in "$@"; do
    envs=(); [ "$s" != base ] && IFS=, read -ra envs <<< "$s"
    env "${envs[@]}" timeout -k 10 120 python -u tools/quick_learner.py humanoid-run 2>&1 | grep -v amdgpu.ids | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$s', d['graph'])" \
      | tee -a "$OUT/ab.txt" || exit 1
  done
done
