# Stall breakdown of the B=32 chain step kernel (microbench chainloop): SQ wait/active split, L1/L2 hit rates
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r74
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/r74/p1 -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 30 > gpurun_out/r74/p1.log 2>&1 || { echo p1 failed; tail gpurun_out/r74/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r74/p2 -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 30 > gpurun_out/r74/p2.log 2>&1 || { echo p2 failed; tail gpurun_out/r74/p2.log; exit 1; }
python tools/pmc_stall.py "chain_kernel<0, 2, 8, 2, 2, true" 524288 gpurun_out/r74/p1/run_counter_collection.csv gpurun_out/r74/p2/run_counter_collection.csv
