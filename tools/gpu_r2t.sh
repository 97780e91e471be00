set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2t
mkdir -p $O
timeout -k 10 300 python -u tools/dump_synth.py 65536 > $O/synth.log 2>&1 || exit $?
cp gpurun_out/synth_65536.npz $O/synth.npz
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
for c in dmtm_drc ch4 synthetic; do timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $O/cfg_$c.log 2>&1 || exit $?; done
