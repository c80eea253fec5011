#!/bin/bash
# GPU box, end of a session: parity suite, smoke, the default bench line, a rocprofv3 kernel trace of the bench,
# and the PMC passes of the dominant kernel (traffic, MFMA busy) merged into profiles/pmc_*.json (args: OUT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
SHORT="--steps 3 --warmup 1 --no-cpu --no-single --no-replay --no-learner --no-icem --no-exact --no-roofline --sweep= --also="
K='wide_step_kernel<4, 7>'
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-single --no-replay --no-learner --no-icem --no-exact --also= > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o run -- python3 bench.py $SHORT > $OUT/pf.log 2>&1 || { tail -5 $OUT/pf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o run -- python3 bench.py $SHORT > $OUT/pw.log 2>&1 || { tail -5 $OUT/pw.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/pm -o run -- python3 bench.py $SHORT > $OUT/pm.log 2>&1 || { tail -5 $OUT/pm.log; exit 1; }
F=$(find $OUT/pf -name '*counter_collection.csv' | head -1); W=$(find $OUT/pw -name '*counter_collection.csv' | head -1); P=$(find $OUT/pm -name '*counter_collection.csv' | head -1)
python3 tools/pmc_traffic.py $F $W "$K" 131072 humanoid-run/B32/wide_step > $OUT/pmc_traffic.txt 2>&1
python3 tools/pmc_mfma.py $P "$K" 131072 humanoid-run/B32/wide_step > $OUT/pmc_mfma.txt 2>&1
cp profiles/pmc_traffic.json profiles/pmc_mfma.json $OUT/
cat $OUT/pmc_traffic.txt $OUT/pmc_mfma.txt
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['learner']['graph'], d['single_env']['value'])"
