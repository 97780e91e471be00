set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2g
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2g/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/bench_configs.py --configs synthetic,dmtm_drc,ch4,cstr --n 16384 --reps 1 --dump > gpurun_out/r2g/cfg.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_configs.py --configs synthetic --n 65536 --reps 1 > gpurun_out/r2g/cfg65k.log 2>&1 || exit $?
