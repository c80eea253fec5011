# HEAD check on a fresh box: GPU parity suite, smoke, then an envs-per-GPU sweep of the humanoid headline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r35
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r35/tests.log 2>&1 || { tail -30 gpurun_out/r35/tests.log; exit 1; }
tail -3 gpurun_out/r35/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r35/smoke.log 2>&1 || { tail -20 gpurun_out/r35/smoke.log; exit 1; }
tail -1 gpurun_out/r35/smoke.log
for b in 1 2 4 8 16 32 64; do
  timeout -k 10 300 python bench.py --envs-per-gpu $b --steps 20 --warmup 3 --no-single --no-replay --no-learner --no-icem --no-cpu > gpurun_out/r35/b$b.json 2> gpurun_out/r35/b$b.err || { echo "FAIL B=$b"; tail -20 gpurun_out/r35/b$b.err; exit 1; }
  echo "B=$b: $(python -c "import json; d=json.loads(open('gpurun_out/r35/b$b.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(d['value'], d['ms_per_step'], d['plan_roofline']['frac_of_fp32_peak'], r.get('frac'))")"
done
