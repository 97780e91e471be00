set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2w
mkdir -p $O
for a in "1024 500" "4096 500"; do timeout -k 10 120 python -u tools/synth_latency.py $a >> $O/lat_main.log 2>&1 || exit $?; done
for a in "1024 500" "4096 500"; do PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_ldspiv.so timeout -k 10 120 python -u tools/synth_latency.py $a >> $O/lat_ldspiv.log 2>&1 || exit $?; done
PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_trace.so PCK_JIT=0 timeout -k 10 120 python -u tools/phase_group.py synthetic 0 > $O/phase_s0.json 2>&1 || exit $?
PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_trace.so PCK_JIT=0 timeout -k 10 120 python -u tools/phase_group.py ch4 500 > $O/phase_ch4.json 2>&1 || exit $?
