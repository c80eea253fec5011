set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/mb/mb_linear 1 && timeout -k 10 120 tools/mb/mb_linear 8
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -T -d gpurun_out/pmc3a -o run --output-format csv -- tools/mb/mb_linear 1 > gpurun_out/pmc3a.log 2>&1; echo "pmc a rc=$?"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_SALU -T -d gpurun_out/pmc3b -o run --output-format csv -- tools/mb/mb_linear 1 > gpurun_out/pmc3b.log 2>&1; echo "pmc b rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace -T -d gpurun_out/kt3 -o run --output-format csv -- tools/mb/mb_linear 1 > gpurun_out/kt3.log 2>&1; echo "kt rc=$?"
ls gpurun_out/pmc3a gpurun_out/pmc3b
