# 16-wave 32-row chain workgroups: parity with TDMPC_CHAIN_NW=16, then B sweep nw 8 vs 16
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r37
export TMPDIR=/tmp
TDMPC_CHAIN_NW=16 timeout -k 10 900 python -u -m pytest tests/test_gpu_plan.py tests/test_icem.py -x -q -m gpu -k "chain32 or bench or graph" --timeout 300 --timeout-method thread > gpurun_out/r37/tests.log 2>&1 || { tail -40 gpurun_out/r37/tests.log; exit 1; }
tail -3 gpurun_out/r37/tests.log
for nw in 16 8; do
for b in 4 8 16; do
  TDMPC_CHAIN_NW=$nw timeout -k 10 300 python bench.py --envs-per-gpu $b --steps 20 --warmup 3 --no-single --no-replay --no-learner --no-icem --no-cpu > gpurun_out/r37/nw${nw}_b$b.json 2> gpurun_out/r37/nw${nw}_b$b.err || { echo "FAIL B=$b"; tail -20 gpurun_out/r37/nw${nw}_b$b.err; exit 1; }
  echo "nw=$nw B=$b: $(python -c "import json; d=json.loads(open('gpurun_out/r37/nw${nw}_b$b.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(d['value'], d['ms_per_step'], d['plan_roofline']['frac_of_fp32_peak'], r.get('frac'), r.get('avg_launch_us'))")"
done
done
