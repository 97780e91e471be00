set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2y
mkdir -p $O
W2=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_w2.so
timeout -k 10 200 python -u tools/dump_synth.py 65536 > $O/main_p1.log 2>&1 || exit $?
PCK_GRP_PASSES=2 timeout -k 10 200 python -u tools/dump_synth.py 65536 > $O/main_p2.log 2>&1 || exit $?
PCK_LIB=$W2 timeout -k 10 200 python -u tools/dump_synth.py 65536 > $O/w2_p1.log 2>&1 || exit $?
PCK_LIB=$W2 PCK_GRP_PASSES=2 timeout -k 10 200 python -u tools/dump_synth.py 65536 > $O/w2_p2.log 2>&1 || exit $?
PCK_LIB=$W2 timeout -k 10 300 python -u bench.py --config ch4 --steps 2 --warmup 1 --no-cpu-baseline > $O/w2_ch4.log 2>&1 || exit $?
PCK_LIB=$W2 timeout -k 10 300 python -u bench.py --config dmtm_drc --steps 2 --warmup 1 --no-cpu-baseline > $O/w2_dmtm.log 2>&1 || exit $?
