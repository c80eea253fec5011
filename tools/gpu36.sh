# chain16 first run: GPU parity suite, then the humanoid headline at B = 2..32 with the row block forced
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r36
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r36/tests.log 2>&1 || { tail -40 gpurun_out/r36/tests.log; exit 1; }
tail -3 gpurun_out/r36/tests.log
for rb in 16 32; do
for b in 2 4 8 16 32; do
  TDMPC_CHAIN_RB=$rb timeout -k 10 300 python bench.py --envs-per-gpu $b --steps 20 --warmup 3 --no-single --no-replay --no-learner --no-icem --no-cpu > gpurun_out/r36/rb${rb}_b$b.json 2> gpurun_out/r36/rb${rb}_b$b.err || { echo "FAIL B=$b"; tail -20 gpurun_out/r36/rb${rb}_b$b.err; exit 1; }
  echo "rb=$rb B=$b: $(python -c "import json; d=json.loads(open('gpurun_out/r36/rb${rb}_b$b.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(d['value'], d['ms_per_step'], d['plan_roofline']['frac_of_fp32_peak'], r.get('frac'), r.get('avg_launch_us'))")"
done
done
