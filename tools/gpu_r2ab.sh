set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2ab
mkdir -p $O
timeout -k 10 200 python -u tools/dump_synth.py 65536 > $O/synth.log 2>&1 || exit $?
cp gpurun_out/synth_65536.npz $O/synth.npz
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py -x -v --timeout 300 --timeout-method thread > $O/gpu_group.txt 2>&1 || exit $?
