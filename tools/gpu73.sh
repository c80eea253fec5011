# x6 default: full GPU suite, smoke, PMC passes of the x6 step kernel, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r73
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r73/tests.log 2>&1 || { tail -40 gpurun_out/r73/tests.log; exit 1; }
tail -1 gpurun_out/r73/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r73/smoke.log 2>&1 || { tail -20 gpurun_out/r73/smoke.log; exit 1; }
tail -1 gpurun_out/r73/smoke.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r73/pmc_fetch -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r73/pmc_fetch.log 2>&1 || { echo pmc1 failed; tail gpurun_out/r73/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r73/pmc_write -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r73/pmc_write.log 2>&1 || { echo pmc2 failed; tail gpurun_out/r73/pmc_write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/r73/pmc_mfma -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r73/pmc_mfma.log 2>&1 || { echo pmc3 failed; tail gpurun_out/r73/pmc_mfma.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/r73/pmc_fetch/run_counter_collection.csv gpurun_out/r73/pmc_write/run_counter_collection.csv "chain_kernel<0, 2, 8, 2, 2, true" 524288 humanoid-run/B32/chain_step_x6 && \
python tools/pmc_mfma.py gpurun_out/r73/pmc_mfma/run_counter_collection.csv "chain_kernel<0, 2, 8, 2, 2, true" 524288 humanoid-run/B32/chain_step_x6 || exit 1
cp profiles/pmc_traffic.json profiles/pmc_mfma.json gpurun_out/r73/
rm -f gpurun_out/r73/pmc_*/run_counter_collection.csv
timeout -k 10 600 python bench.py > gpurun_out/r73/bench.json 2> gpurun_out/r73/bench.err || { tail -30 gpurun_out/r73/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r73/bench.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['roofline'])); print(d['plan_roofline'], d['exact_f32_mfma'], d['batch_sweep'], d['single_env']['value'], d['icem']['ms_per_step'], d['icem']['batch32']['value'])"
