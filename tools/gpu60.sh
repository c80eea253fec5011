set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r60
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_learner.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r60/tests.log 2>&1 || { tail -40 gpurun_out/r60/tests.log; exit 1; }
tail -1 gpurun_out/r60/tests.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-single --no-replay --no-roofline --sweep "" --no-cpu > gpurun_out/r60/bench.json 2> gpurun_out/r60/bench.err || { tail -30 gpurun_out/r60/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r60/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['learner'])); print(json.dumps(d['icem']))"
