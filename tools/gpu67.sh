set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in humanoid-run-l512 humanoid-run; do timeout -k 10 120 python tools/quick_time.py $c 1 2>&1 | grep plan-steps; done
