set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit 1
for v in 1 2; do TDMPC_LDS_VARIANT=$v timeout -k 10 120 tools/mb/mb_linear 8 > gpurun_out/mb_v$v.log 2>&1 || exit 1; echo "lds variant $v"; sed -n 1,8p gpurun_out/mb_v$v.log; done
timeout -k 10 400 python bench.py > gpurun_out/bench_r01b.json 2> gpurun_out/bench_r01b.err || { echo bench failed; tail -20 gpurun_out/bench_r01b.err; exit 1; }
cat gpurun_out/bench_r01b.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || { echo prof failed; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- tools/mb/mb_linear 8 s2loop 50 > gpurun_out/pmc_fetch.log 2>&1 || { echo pmc1 failed; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- tools/mb/mb_linear 8 s2loop 50 > gpurun_out/pmc_write.log 2>&1 || { echo pmc2 failed; exit 1; }
echo ALLDONE
