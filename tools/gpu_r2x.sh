set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2x
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --scaling weak --no-cpu-baseline > $O/bench_weak.log 2>&1 || exit $?
for a in "1024 500" "4096 500"; do timeout -k 10 120 python -u tools/synth_latency.py $a >> $O/lat_main.log 2>&1 || exit $?; done
for a in "1024 500" "4096 500"; do PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_ldspiv.so timeout -k 10 120 python -u tools/synth_latency.py $a >> $O/lat_ldspiv.log 2>&1 || exit $?; done
PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_trace.so PCK_JIT=0 timeout -k 10 120 python -u tools/phase_group.py synthetic 0 > $O/phase_s0.json 2>&1 || exit $?
