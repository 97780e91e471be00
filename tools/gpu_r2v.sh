set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r2t.sh || exit $?
bash tools/gpu_r2u.sh || exit $?
