set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab
S="--steps 30 --warmup 5 --no-cpu --no-single --no-replay --no-learner --no-icem --no-exact --no-roofline --sweep= --also="
for r in 1 2; do
  for k in base TDMPC_CHAIN_IL=1 TDMPC_CHAIN_XCD=1; do
    if [ $k = base ]; then E=""; else E="$k"; fi
    env $E timeout -k 10 180 python bench.py $S > gpurun_out/ab/$k.$r.json 2> gpurun_out/ab/$k.$r.err || exit 1
    echo "$k $r $(python3 -c "import json;d=json.load(open('gpurun_out/ab/$k.$r.json'));print(d['value'],d['ms_per_step'])")"
  done
done
