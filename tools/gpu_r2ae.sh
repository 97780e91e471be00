set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2ae
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
for c in ch4 dmtm_drc synthetic; do timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 > $O/cfg_$c.log 2>&1 || exit $?; done
