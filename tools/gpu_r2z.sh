set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2z
mkdir -p $O
PCK_JIT=0 PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_trace.so MAXSTEPS=200000 timeout -k 10 200 python -u tools/trace_group.py 39547 > $O/trace.log 2>&1 || exit $?
