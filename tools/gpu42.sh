# horizon-batched learner: GPU parity + learner bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r42
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_learner.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r42/tests.log 2>&1 || { tail -40 gpurun_out/r42/tests.log; exit 1; }
tail -2 gpurun_out/r42/tests.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-single --no-replay --no-icem --no-roofline --sweep "" > gpurun_out/r42/bench.json 2> gpurun_out/r42/bench.err || { tail -30 gpurun_out/r42/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r42/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['learner']))"
