set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r46
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_learner.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r46/tests.log 2>&1 || { tail -40 gpurun_out/r46/tests.log; exit 1; }
tail -2 gpurun_out/r46/tests.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-single --no-replay --no-icem --no-roofline --sweep "" --no-cpu > gpurun_out/r46/bench.json 2> gpurun_out/r46/bench.err || { tail -30 gpurun_out/r46/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r46/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['learner']))"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r46/kt -o run --output-format csv -- python tools/learner_trace.py > gpurun_out/r46/kt.log 2>&1 || { tail gpurun_out/r46/kt.log; exit 1; }
python tools/learner_prof.py gpurun_out/r46/kt/run_kernel_trace.csv 10 > gpurun_out/r46/learner.txt
rm -f gpurun_out/r46/kt/run_kernel_trace.csv
head -20 gpurun_out/r46/learner.txt
