set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err; echo "bench rc=$?"; cat gpurun_out/bench_r01.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-single --no-roofline > gpurun_out/prof_bench.log 2>&1; echo "prof rc=$?"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-single --no-roofline --no-graph > gpurun_out/pmc_fetch.log 2>&1; echo "pmc fetch rc=$?"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-single --no-roofline --no-graph > gpurun_out/pmc_write.log 2>&1; echo "pmc write rc=$?"
