# chain threshold for small batches (chain16 makes 1-2 env launches wider): B = 1, 2, 4 at several TDMPC_CHAIN_WGS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r38
export TMPDIR=/tmp
for w in 128 64 32 16; do
for b in 1 2 4 8; do
  TDMPC_CHAIN_WGS=$w timeout -k 10 300 python bench.py --envs-per-gpu $b --steps 20 --warmup 3 --no-single --no-replay --no-learner --no-icem --no-cpu --no-roofline > gpurun_out/r38/w${w}_b$b.json 2> gpurun_out/r38/w${w}_b$b.err || { echo "FAIL B=$b"; tail -20 gpurun_out/r38/w${w}_b$b.err; exit 1; }
  echo "wgs=$w B=$b: $(python -c "import json; d=json.loads(open('gpurun_out/r38/w${w}_b$b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['plan_roofline']['frac_of_fp32_peak'])")"
done
done
