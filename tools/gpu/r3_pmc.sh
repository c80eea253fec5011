#!/bin/bash
# PMC passes over the humanoid B=32 plan (quick_time.py), wide step kernel on; one counter set per rocprofv3 run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3pmc}
mkdir -p $O
export TMPDIR=/tmp TDMPC_WIDE=1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python -u tools/quick_time.py humanoid-run 32 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  f=$(find $O/p$i -name '*counter_collection.csv' | head -1)
  python tools/pmc_stall.py wide_step_kernelILi4ELi7 131072 $f > $O/p$i.txt && cat $O/p$i.txt
done
