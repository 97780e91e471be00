set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2a
PCK_LIB=pycatkin_amd/_ab/lib_trace.so MAXSTEPS=200000 timeout -k 10 240 python -u tools/trace_group.py 1 659 888 > gpurun_out/r2a/trace.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2a/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r2a/bench.log 2>&1 || exit $?
for r in 0 3 7; do timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --emulate $r/8 --no-cpu-baseline > gpurun_out/r2a/emul_$r.log 2>&1 || exit $?; done
