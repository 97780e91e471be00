set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2p
mkdir -p $O
for a in "1 500" "1024 500" "4096 500"; do timeout -k 10 120 python -u tools/synth_latency.py $a >> $O/lat.log 2>&1 || exit $?; done
PCK_JIT=0 timeout -k 10 120 python -u tools/synth_latency.py 1024 500 >> $O/lat.log 2>&1 || exit $?
export PCK_JIT=0 PCK_LIB=pycatkin_amd/_ab/lib_trace.so
timeout -k 10 120 python -u tools/phase_group.py synthetic 0 > $O/phase_s0.json 2>&1 || exit $?
timeout -k 10 120 python -u tools/phase_group.py dmtm 500 > $O/phase_dmtm.json 2>&1 || exit $?
