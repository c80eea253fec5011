set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit 1
for v in 0 5; do echo "variant $v"; TDMPC_THR_VARIANT=$v timeout -k 10 120 tools/mb/mb_linear 8 || exit 1; done
echo "B=32"; timeout -k 10 120 tools/mb/mb_linear 32
