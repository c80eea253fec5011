# Snapshot: full GPU suite, smoke, default bench, rocprof stats, every config
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r76/cfg
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r76/tests.log 2>&1 || { tail -40 gpurun_out/r76/tests.log; exit 1; }
tail -1 gpurun_out/r76/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r76/smoke.log 2>&1 || { tail -20 gpurun_out/r76/smoke.log; exit 1; }
tail -1 gpurun_out/r76/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r76/bench.json 2> gpurun_out/r76/bench.err || { tail -30 gpurun_out/r76/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r76/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline'].get('mfma_util_pmc'), d['roofline'].get('hbm_frac_pmc'), d['batch_sweep'], d['single_env']['value'], d['learner']['graph'], d['icem']['ms_per_step'], d['icem']['batch32']['value'], d['replay_sampler']['with_replacement']['us_per_sample'], d['cpu_baseline']['value'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r76/prof -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/r76/prof.log 2>&1 || { tail gpurun_out/r76/prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/r76/prof/run_kernel_trace.csv > gpurun_out/r76/prof_summary.txt
rm -f gpurun_out/r76/prof/run_kernel_trace.csv
for c in cheetah-run humanoid-run-l512 dog-run quadruped-run-pixels; do
  timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 3 --no-replay --no-learner --no-icem --cpu-budget 10 > gpurun_out/r76/cfg/$c.json 2> gpurun_out/r76/cfg/$c.err || { echo "FAIL $c"; tail -20 gpurun_out/r76/cfg/$c.err; exit 1; }
  echo "$c: $(python -c "import json,sys; d=json.loads(open('gpurun_out/r76/cfg/$c.json').read().strip().splitlines()[-1]); print(d['value'], d['plan_roofline']['frac_of_fp32_peak'], d['roofline']['frac'], d['batch_sweep']['8']['value'], d['single_env']['value'], d['cpu_baseline']['value'])")"
done
echo ALLDONE
