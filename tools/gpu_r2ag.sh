set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2ag
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit $?
for c in ch4 dmtm_drc; do timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/def_$c.log 2>&1 || exit $?; done
for c in ch4 dmtm_drc; do PCK_GRP_DEGMAX=1 timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/deg_$c.log 2>&1 || exit $?; done
PCK_GRP_DEGMAX=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py -x -q --timeout 300 --timeout-method thread > $O/deg_group.txt 2>&1 || exit $?
