#!/bin/bash
# Every GPU-box procedure of this repo, one stage per argument, run in order; the first failing stage ends the call.
#   tools/gpu/suite.sh OUT STAGE [STAGE ...]
# Stages (results under gpurun_out/OUT/):
#   tests            the whole `pytest -m gpu` suite
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (bench.json)
#   prof             rocprofv3 kernel trace of a short bench run, summarised by kernel and grid (prof_summary.txt)
#   pmc              PMC passes of the dominant kernel (FETCH_SIZE, WRITE_SIZE, MFMA busy), merged into
#                    profiles/pmc_traffic.json / pmc_mfma.json copies under OUT
#   stall            SQ stall / instruction-mix passes of the wide step kernel (pmc_stall.py)
#   pytest:EXPR      the GPU plan / config / sharded tests selected by -k EXPR
#   ab:VAR=v1,v2     alternating runs of tools/quick_time.py (CONFIG, ENVS below) with VAR at each value
#   lib:v1,v2        the same with TDMPC_LIB_PATH=tdmpc_amd/libtdmpc_hip_<v>.so (python -m tdmpc_amd.build --variant)
#   single:v1,v2     literal single-env plan() per library variant (6 rounds of 150 calls, median per variant)
#   stamps           per-step shader stamps of the wide step kernel (needs the `ws` variant: -DWS_STAMPS)
#   learner:VAR=v1,v2  the learner / train-loop / adam tests, then an A/B of VAR on the humanoid update time
#   lab:VAR=v1,v2    the humanoid update-time A/B of `learner:` without its tests
#   labs:A=1 B=2|A=0 the same over whole environment settings ('|' between settings)
#   lgbench          lg_gemm tile timings of the learner's products (tools/lg_gemm_bench.py)
#   p1stamps         per-hand-off timeline of the one-env persistent plan (tools/p1_stamps.py)
#   qt               tools/quick_time.py on CONFIG / ENVS (qt.txt)
#   trace            per-kernel breakdown of one plan of CONFIG / ENVS (rocprofv3 kernel trace, tools/plan_trace.py)
#   ringpmc          SQ counter passes of the LDS-DMA ring probe's cases (tools/mb/dma_ring)
# Environment: CONFIG (default humanoid-run), ENVS (default 32).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
CONFIG=${CONFIG:-humanoid-run}; ENVS=${ENVS:-32}
SHORT="--steps 3 --warmup 1 --no-cpu --no-single --no-replay --no-learner --no-icem --no-exact --no-roofline --sweep= --also="
WK='wide_step_kernel<4, 7, 0>'

for stage in "$@"; do
  case $stage in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
      tail -1 "$OUT/tests.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { tail -20 "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_us'])" ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 3 \
        --no-cpu --no-single --no-replay --no-learner --no-icem --no-exact --also= > "$OUT/prof.log" 2>&1 \
        || { tail -20 "$OUT/prof.log"; exit 1; }
      python3 tools/rocpd_summary.py "$OUT/prof/run_results.db" 16 --grid > "$OUT/prof_summary.txt" 2>&1
      cut -c1-150 "$OUT/prof_summary.txt" | head -12 ;;
    pmc)
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pf" -o run -- python3 bench.py $SHORT > "$OUT/pf.log" 2>&1 || { tail -5 "$OUT/pf.log"; exit 1; }
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pw" -o run -- python3 bench.py $SHORT > "$OUT/pw.log" 2>&1 || { tail -5 "$OUT/pw.log"; exit 1; }
      timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d "$OUT/pm" -o run -- python3 bench.py $SHORT > "$OUT/pm.log" 2>&1 || { tail -5 "$OUT/pm.log"; exit 1; }
      F=$(find "$OUT/pf" -name '*counter_collection.csv' | head -1); W=$(find "$OUT/pw" -name '*counter_collection.csv' | head -1)
      P=$(find "$OUT/pm" -name '*counter_collection.csv' | head -1)
      python3 tools/pmc_traffic.py "$F" "$W" "$WK" 131072 humanoid-run/B32/wide_step > "$OUT/pmc_traffic.txt" 2>&1
      python3 tools/pmc_mfma.py "$P" "$WK" 131072 humanoid-run/B32/wide_step > "$OUT/pmc_mfma.txt" 2>&1
      cp profiles/pmc_traffic.json profiles/pmc_mfma.json "$OUT/"
      cat "$OUT/pmc_traffic.txt" "$OUT/pmc_mfma.txt" ;;
    stall)
      P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
      P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
      i=0
      for P in "$P1" "$P2"; do
        i=$((i+1))
        timeout -s KILL 150 rocprofv3 --pmc $P -d "$OUT/s$i" -o run --output-format csv -- python -u tools/quick_time.py humanoid-run 32 \
          > "$OUT/s$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/s$i.log"; exit 1; }
        f=$(find "$OUT/s$i" -name '*counter_collection.csv' | head -1)
        python tools/pmc_stall.py "wide_step_kernel<4, 7>" 131072 "$f" > "$OUT/s$i.txt" && cat "$OUT/s$i.txt"
      done ;;
    ringpmc)
      # the LDS-DMA ring probe's cases (tools/mb/dma_ring.hip: the wide step kernel's ring without its arithmetic),
      # two SQ counter passes each: where the MFMA + DMA serialisation waits
      R1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
      R2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
      timeout -k 10 60 tools/mb/dma_ring 94 2304 > "$OUT/ring_times.txt" 2>&1 || { tail -5 "$OUT/ring_times.txt"; exit 1; }
      cat "$OUT/ring_times.txt"
      for c in mfma mfma_lds mfma_dma full dma; do
        i=0
        for P in "$R1" "$R2"; do
          i=$((i+1))
          timeout -s KILL 60 rocprofv3 --pmc $P -d "$OUT/r_$c$i" -o run --output-format csv -- tools/mb/dma_ring 94 2304 $c \
            > "$OUT/r_$c$i.log" 2>&1 || { echo "ring pass $c $i failed"; tail -5 "$OUT/r_$c$i.log"; exit 1; }
          f=$(find "$OUT/r_$c$i" -name '*counter_collection.csv' | head -1)
          echo "== $c pass $i"; python tools/pmc_stall.py ring_kernel 131072 "$f" | tee "$OUT/r_$c$i.txt"
        done
      done ;;
    pytest:*)
      timeout -k 10 500 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_configs.py tests/test_gpu_sharded.py -m gpu -v -x \
        --timeout 200 --timeout-method thread -k "${stage#pytest:}" > "$OUT/tests_sel.txt" 2>&1 \
        || { echo "tests failed"; tail -40 "$OUT/tests_sel.txt"; exit 1; }
      grep -E "passed|failed" "$OUT/tests_sel.txt" | tail -1 ;;
    ab:*)
      kv=${stage#ab:}; var=${kv%%=*}; vals=${kv#*=}
      for i in 1 2 3; do
        for v in ${vals//,/ }; do
          env "$var=$v" timeout -k 10 120 python -u tools/quick_time.py "$CONFIG" "$ENVS" 2>&1 | grep -v amdgpu.ids \
            | sed "s/^/$var=$v: /" || exit 1
        done
      done ;;
    lib:*)
      for i in 1 2 3; do
        for v in $(echo "${stage#lib:}" | tr , ' '); do
          TDMPC_LIB_PATH=$PWD/tdmpc_amd/libtdmpc_hip_$v.so timeout -k 10 120 python -u tools/quick_time.py "$CONFIG" "$ENVS" \
            2>&1 | grep -v amdgpu.ids | sed "s/^/$v: /" || exit 1
        done
      done ;;
    single:*)
      tmp=$(mktemp)
      for i in 1 2 3 4 5 6; do
        for v in $(echo "${stage#single:}" | tr , ' '); do
          TDMPC_LIB_PATH=$PWD/tdmpc_amd/libtdmpc_hip_$v.so timeout -k 10 120 python -u tools/single_time.py humanoid-run 150 2>&1 \
            | grep -v amdgpu.ids | sed "s/^/$v: /" | tee -a "$tmp" || exit 1
        done
      done
      python3 - "$tmp" <<'PY'
import re, statistics, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"(\S+): plan\(\) single env: ([0-9.]+) ms", line)
    if m: d[m.group(1)].append(float(m.group(2)))
for v, xs in d.items():
    print(f"{v}: median {statistics.median(xs):.4f} ms/call ({1e3 / statistics.median(xs):.1f} plan-steps/s), min {min(xs):.4f}, n={len(xs)}")
PY
      ;;
    stamps)
      TDMPC_LIB_PATH=$PWD/tdmpc_amd/libtdmpc_hip_ws.so timeout -k 10 200 python -u tools/ws_stamps.py 32 \
        > "$OUT/stamps.txt" 2>&1 || exit 1
      grep -v amdgpu.ids "$OUT/stamps.txt" | head -5 ;;
    learner:*)
      kv=${stage#learner:}; var=${kv%%=*}; vals=${kv#*=}
      timeout -k 10 600 python -u -m pytest tests/test_learner.py tests/test_gpu_train_loop.py tests/test_gpu_adam.py -m gpu -v -x \
        --timeout 300 --timeout-method thread > "$OUT/learner_tests.txt" 2>&1 || { echo "tests failed"; tail -40 "$OUT/learner_tests.txt"; exit 1; }
      grep -E "passed|failed" "$OUT/learner_tests.txt" | tail -1
      for i in 1 2 3; do
        for v in ${vals//,/ }; do
          env "$var=$v" timeout -k 10 120 python -u tools/quick_learner.py humanoid-run 2>&1 | grep -v amdgpu.ids | \
            python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$var=$v', d['graph'])" || exit 1
        done
      done ;;
    lab:*)
      kv=${stage#lab:}; var=${kv%%=*}; vals=${kv#*=}
      for i in 1 2 3; do
        for v in ${vals//,/ }; do
          env "$var=$v" timeout -k 10 120 python -u tools/quick_learner.py humanoid-run 2>&1 | grep -v amdgpu.ids | \
            python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$var=$v', d['graph'])" || exit 1
        done
      done ;;
    labs:*)   # labs:A=1 B=2|A=0 -- the update-time A/B over whole environment settings ('|' between settings)
      sets=${stage#labs:}
      for i in 1 2 3; do
        IFS='|' read -ra arr <<< "$sets"
        for st in "${arr[@]}"; do
          env $st timeout -k 10 120 python -u tools/quick_learner.py humanoid-run 2>&1 | grep -v amdgpu.ids | \
            python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$st', d['graph'])" || exit 1
        done
      done ;;
    lgbench*)
      timeout -k 10 200 python -u tools/lg_gemm_bench.py ${stage#lgbench} > "$OUT/lg_gemm.txt" 2>&1 || { tail -20 "$OUT/lg_gemm.txt"; exit 1; }
      grep -v amdgpu.ids "$OUT/lg_gemm.txt" | tail -30 ;;
    p1stamps)
      timeout -k 10 120 python -u tools/p1_stamps.py "$CONFIG" > "$OUT/p1_stamps.txt" 2>&1 || { tail -20 "$OUT/p1_stamps.txt"; exit 1; }
      tail -4 "$OUT/p1_stamps.txt" ;;
    trace)
      # per-kernel breakdown of one plan of CONFIG / ENVS (rocprofv3 kernel trace of tools/quick_time.py, eager-free
      # graph replays; tools/plan_trace.py summarises the last complete plan)
      timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run -- python -u tools/quick_time.py "$CONFIG" "$ENVS" \
        > "$OUT/tr.log" 2>&1 || { tail -20 "$OUT/tr.log"; exit 1; }
      f=$(find "$OUT/tr" -name '*kernel_trace.csv' | head -1)
      python3 tools/plan_trace.py "$f" > "$OUT/plan_trace_${CONFIG}_b${ENVS}.txt" 2>&1; cat "$OUT/plan_trace_${CONFIG}_b${ENVS}.txt" ;;
    qt)
      timeout -k 10 120 python -u tools/quick_time.py "$CONFIG" "$ENVS" > "$OUT/qt.txt" 2>&1 || { tail -20 "$OUT/qt.txt"; exit 1; }
      grep -v amdgpu.ids "$OUT/qt.txt" ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
