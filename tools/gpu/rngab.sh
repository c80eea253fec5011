#!/bin/bash
# GPU box: reference-order draw kernel parity, then the bench's plan line with rng=fused vs rng=reference
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rngab
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "reference_normals or reference_draws or rng_order" > gpurun_out/rngab/tests.log 2>&1 || { tail -40 gpurun_out/rngab/tests.log; exit 1; }
tail -2 gpurun_out/rngab/tests.log
F="--no-cpu --no-roofline --no-single --no-replay --no-learner --no-icem --no-exact --also= --sweep="
for r in fused reference fused reference; do
  timeout -k 10 200 python bench.py $F --rng $r 2>/dev/null | tail -1 > gpurun_out/rngab/$r.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/rngab/$r.json'));print('$r',d['value'],d['ms_per_step'])"
done
