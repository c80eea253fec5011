# Snapshot (x6 mode 3 default): full GPU suite, smoke, PMC passes of the step kernel, default bench, rocprof, configs
set -o pipefail
cd $GRAFT_REPO_ROOT
R=gpurun_out/r91
mkdir -p $R/cfg
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 1; }
tail -1 $R/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || { tail -20 $R/smoke.log; exit 1; }
tail -1 $R/smoke.log
K="chain_kernel<0, 4, 4, 2, 2, 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/pmc_fetch -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > $R/pmc_fetch.log 2>&1 || { echo pmc1 failed; tail $R/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/pmc_write -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > $R/pmc_write.log 2>&1 || { echo pmc2 failed; tail $R/pmc_write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $R/pmc_mfma -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > $R/pmc_mfma.log 2>&1 || { echo pmc3 failed; tail $R/pmc_mfma.log; exit 1; }
python tools/pmc_traffic.py $R/pmc_fetch/run_counter_collection.csv $R/pmc_write/run_counter_collection.csv "$K" 262144 humanoid-run/B32/chain_step_x6 && \
python tools/pmc_mfma.py $R/pmc_mfma/run_counter_collection.csv "$K" 262144 humanoid-run/B32/chain_step_x6 || exit 1
cp profiles/pmc_traffic.json profiles/pmc_mfma.json $R/
rm -f $R/pmc_*/run_counter_collection.csv
timeout -k 10 600 python bench.py > $R/bench.json 2> $R/bench.err || { tail -30 $R/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$R/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['frac_of_fp32_mfma_peak'], d['roofline'].get('mfma_util_pmc'), d['exact_f32_mfma']['value'], d['batch_sweep'], d['single_env']['value'], d['learner']['graph'], d['icem']['ms_per_step'], d['icem']['batch32']['value'], d['replay_sampler']['with_replacement']['us_per_sample'], d['cpu_baseline']['value'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/prof -o run --output-format csv -- python bench.py --no-cpu > $R/prof.log 2>&1 || { tail $R/prof.log; exit 1; }
python tools/prof_summary.py $R/prof/run_kernel_trace.csv > $R/prof_summary.txt
rm -f $R/prof/run_kernel_trace.csv
for c in cheetah-run humanoid-run-l512 dog-run quadruped-run-pixels; do
  timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 3 --no-replay --no-learner --no-icem --cpu-budget 10 > $R/cfg/$c.json 2> $R/cfg/$c.err || { echo "FAIL $c"; tail -20 $R/cfg/$c.err; exit 1; }
  echo "$c: $(python -c "import json,sys; d=json.loads(open('$R/cfg/$c.json').read().strip().splitlines()[-1]); print(d['value'], d['exact_f32_mfma']['value'], d['plan_roofline']['frac_of_fp32_peak'], d['roofline']['frac'], d['roofline']['frac_of_fp32_mfma_peak'], d['batch_sweep']['8']['value'], d['single_env']['value'], d['cpu_baseline']['value'])")"
done
echo ALLDONE
