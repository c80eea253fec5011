# Round snapshot: full bench (default B = 32) + rocprof kernel stats + PMC traffic / MFMA passes + every config
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r53/cfg
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r53/pmc_fetch -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r53/pmc_fetch.log 2>&1 || { echo pmc1 failed; tail gpurun_out/r53/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r53/pmc_write -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r53/pmc_write.log 2>&1 || { echo pmc2 failed; tail gpurun_out/r53/pmc_write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/r53/pmc_mfma -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r53/pmc_mfma.log 2>&1 || { echo pmc3 failed; tail gpurun_out/r53/pmc_mfma.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/r53/pmc_fetch/run_counter_collection.csv gpurun_out/r53/pmc_write/run_counter_collection.csv "chain_kernel<0, 2" 524288 humanoid-run/B32/chain_step
python tools/pmc_mfma.py gpurun_out/r53/pmc_mfma/run_counter_collection.csv "chain_kernel<0, 2" 524288 humanoid-run/B32/chain_step
rm -f gpurun_out/r53/pmc_*/run_counter_collection.csv
timeout -k 10 600 python bench.py > gpurun_out/r53/bench.json 2> gpurun_out/r53/bench.err || { tail -30 gpurun_out/r53/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r53/bench.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['roofline']), d['batch_sweep'], d['single_env']['value'], d['learner']['graph'], d['icem']['ms_per_step'], d['cpu_baseline']['value'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r53/prof -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/r53/prof.log 2>&1 || { tail gpurun_out/r53/prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/r53/prof/run_kernel_trace.csv > gpurun_out/r53/prof_summary.txt
rm -f gpurun_out/r53/prof/run_kernel_trace.csv
for c in cheetah-run humanoid-run-l512 dog-run quadruped-run-pixels; do
  timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 3 --no-replay --no-learner --no-icem --cpu-budget 10 > gpurun_out/r53/cfg/$c.json 2> gpurun_out/r53/cfg/$c.err || { echo "FAIL $c"; tail -20 gpurun_out/r53/cfg/$c.err; exit 1; }
  echo "$c: $(python -c "import json,sys; d=json.loads(open('gpurun_out/r53/cfg/$c.json').read().strip().splitlines()[-1]); print(d['value'], d['plan_roofline']['frac_of_fp32_peak'], d['roofline']['frac'], d['batch_sweep'], d['single_env']['value'], d['cpu_baseline']['value'])")"
done
echo ALLDONE
