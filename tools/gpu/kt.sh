#!/bin/bash
# GPU box: rocprofv3 kernel trace of tools/quick_time.py (args: OUT config B [ENV=VAL ...]); summary -> OUT/summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; CFG=$2; B=$3; shift 3
mkdir -p $OUT
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/quick_time.py $CFG $B > $OUT/log.txt 2>&1 || { tail -5 $OUT/log.txt; exit 1; }
python3 tools/rocpd_summary.py $OUT/prof/run_results.db 14 > $OUT/summary.txt
grep plan-steps $OUT/log.txt
cat $OUT/summary.txt
