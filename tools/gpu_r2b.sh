set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2b
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2b/gpu_group.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/bench_configs.py --configs synthetic,dmtm_drc,ch4 --n 16384 --reps 1 --dump > gpurun_out/r2b/cfg.log 2>&1 || exit $?
