set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu/stamps.sh st2 && tools/gpu/learner_ab.sh lg1 TDMPC_LG_BLAS "1 0"
