# LDS-only barriers in the chain kernels: parity, stamps, headline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r48
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r48/tests.log 2>&1 || { tail -40 gpurun_out/r48/tests.log; exit 1; }
tail -2 gpurun_out/r48/tests.log
timeout -k 10 200 tools/mb/mb_linear_st 8 > gpurun_out/r48/st8.log 2>&1 || { tail -20 gpurun_out/r48/st8.log; exit 1; }
grep -A1 "chain" gpurun_out/r48/st8.log | grep -v blockIdx
timeout -k 10 200 tools/mb/mb_linear_st 32 > gpurun_out/r48/st32.log 2>&1 || { tail -20 gpurun_out/r48/st32.log; exit 1; }
grep -A1 "chain" gpurun_out/r48/st32.log | grep -v blockIdx
for b in 8 32; do
  timeout -k 10 300 python bench.py --envs-per-gpu $b --steps 20 --warmup 3 --no-single --no-replay --no-learner --no-icem --no-cpu --sweep "" > gpurun_out/r48/b$b.json 2> gpurun_out/r48/b$b.err || { echo "FAIL B=$b"; tail -20 gpurun_out/r48/b$b.err; exit 1; }
  echo "B=$b: $(python -c "import json; d=json.loads(open('gpurun_out/r48/b$b.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(d['value'], d['ms_per_step'], d['plan_roofline']['frac_of_fp32_peak'], r.get('frac'), r.get('avg_launch_us'))")"
done
