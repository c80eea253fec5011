# final check of the committed build: full GPU suite, smoke, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
R=gpurun_out/r93
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || { tail -40 $R/tests.log; exit 1; }
tail -1 $R/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || { tail -20 $R/smoke.log; exit 1; }
tail -1 $R/smoke.log
timeout -k 10 600 python bench.py > $R/bench.json 2> $R/bench.err || { tail -30 $R/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$R/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['exact_f32_mfma']['value'], d['batch_sweep']['8']['value'], d['single_env']['value'], d['cpu_baseline']['value'])"
