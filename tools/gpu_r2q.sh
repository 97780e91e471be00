set -o pipefail
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/ab/summary.txt
bash tools/ab_run.sh cur v2 noall v2 cur || exit $?
