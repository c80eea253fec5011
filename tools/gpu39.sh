# Full bench at the new default (B = 32 envs per GPU) + rocprof kernel stats of the same command + PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r39
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/r39/bench.json 2> gpurun_out/r39/bench.err || { tail -30 gpurun_out/r39/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r39/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['plan_roofline'], d['batch_sweep'], d['single_env']['value'], d['cpu_baseline'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r39/prof -o run --output-format csv -- python bench.py --no-cpu --no-replay --no-learner --no-icem > gpurun_out/r39/prof.log 2>&1 || { tail gpurun_out/r39/prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/r39/prof/run_kernel_trace.csv > gpurun_out/r39/prof_summary.txt
rm -f gpurun_out/r39/prof/run_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r39/qt -o run --output-format csv -- python tools/quick_time.py humanoid-run 32 > gpurun_out/r39/qt.log 2>&1 || { tail gpurun_out/r39/qt.log; exit 1; }
python tools/plan_trace.py gpurun_out/r39/qt/run_kernel_trace.csv 1 > gpurun_out/r39/plan_b32.txt || true
rm -f gpurun_out/r39/qt/run_kernel_trace.csv
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r39/pmc_fetch -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r39/pmc_fetch.log 2>&1 || { echo pmc1 failed; tail gpurun_out/r39/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r39/pmc_write -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r39/pmc_write.log 2>&1 || { echo pmc2 failed; tail gpurun_out/r39/pmc_write.log; exit 1; }
ls gpurun_out/r39/pmc_fetch gpurun_out/r39/pmc_write
echo ALLDONE
