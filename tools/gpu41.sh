# MFMA utilisation of the dominant chain step kernel (B = 32): SQ_VALU_MFMA_BUSY_CYCLES against GRBM_GUI_ACTIVE
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r41
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r41/avail.txt 2>&1 || true
grep -i -E "MFMA|GRBM_GUI_ACTIVE|SQ_BUSY_CYCLES|SQ_WAVE_CYCLES" gpurun_out/r41/avail.txt | head -30
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/r41/pmc_mfma -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r41/pmc_mfma.log 2>&1 || { echo pmc failed; tail gpurun_out/r41/pmc_mfma.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace -d gpurun_out/r41/kt -o run --output-format csv -- tools/mb/mb_linear 32 chainloop 50 > gpurun_out/r41/kt.log 2>&1 || { echo kt failed; tail gpurun_out/r41/kt.log; exit 1; }
ls gpurun_out/r41/pmc_mfma gpurun_out/r41/kt
echo ALLDONE
