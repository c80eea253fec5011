#!/bin/bash
# Round 3 iteration loop for the wide step kernel: parity subset (stop on failure), A/B timing, rocprof by grid.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3q}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_configs.py -v -x --timeout 200 --timeout-method thread \
    -k "wide or bench_shape or inf_hidden" > $O/wide_tests.txt 2>&1 || { echo "wide tests failed"; tail -30 $O/wide_tests.txt; exit 1; }
tail -1 $O/wide_tests.txt
for i in 1 2; do
  for w in 0 1; do
    TDMPC_WIDE=$w timeout -k 10 120 python -u tools/quick_time.py humanoid-run 32 >> $O/ab.txt 2>&1 || exit 1
    echo "  (TDMPC_WIDE=$w)" >> $O/ab.txt
  done
done
export TMPDIR=/tmp
TDMPC_WIDE=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u tools/quick_time.py humanoid-run 32 > $O/prof.log 2>&1 || exit 1
python tools/rocpd_summary.py $O/prof/run_results.db 8 --grid > $O/prof_summary.txt 2>&1
grep -v amdgpu.ids $O/ab.txt
cut -c1-140 $O/prof_summary.txt
if [ -f tdmpc_amd/libtdmpc_hip_ws.so ]; then
  TDMPC_WIDE=1 TDMPC_LIB_PATH=$PWD/tdmpc_amd/libtdmpc_hip_ws.so timeout -k 10 200 python -u tools/ws_stamps.py 32 > $O/stamps.txt 2>&1 && grep -v amdgpu.ids $O/stamps.txt
fi
