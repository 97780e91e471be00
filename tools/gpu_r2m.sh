set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2m
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit $?
bash tools/profile.sh r2m/prof_volcano python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $?
