set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2r
mkdir -p $O
rm -f gpurun_out/ab/summary.txt
bash tools/ab_run.sh cur pos1 pos0 pos1 cur || exit $?
PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_pos0.so timeout -k 10 300 python -u tools/dump_synth.py 65536 > $O/synth_pos0.log 2>&1 || exit $?
PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_pos0.so timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_pos0.txt 2>&1 || exit $?
