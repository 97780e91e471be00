set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py -x -v --timeout 300 --timeout-method thread -k "stragglers or patched_rate" > $O/t.txt 2>&1 || exit $?
