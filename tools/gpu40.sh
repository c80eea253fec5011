# Every GPU config of the scope table at the default 32 envs per GPU (and the 8-per-GPU batch in the same run)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg40
export TMPDIR=/tmp
for c in humanoid-run cheetah-run humanoid-run-l512 dog-run quadruped-run-pixels; do
  timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 3 --no-replay --no-learner --no-icem --cpu-budget 10 > gpurun_out/cfg40/$c.json 2> gpurun_out/cfg40/$c.err || { echo "FAIL $c"; tail -20 gpurun_out/cfg40/$c.err; exit 1; }
  echo "$c: $(python -c "import json,sys; d=json.loads(open('gpurun_out/cfg40/$c.json').read().strip().splitlines()[-1]); print(d['value'], d['plan_roofline']['frac_of_fp32_peak'], d['roofline']['frac'], d['batch_sweep'], d['single_env']['value'], d['cpu_baseline']['value'])")"
done
