set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/phase2
export PCK_JIT=0
for v in trace trace_lds; do
  export PCK_LIB=pycatkin_amd/_ab/lib_$v.so
  timeout -k 10 120 python -u tools/phase_group.py synthetic 0 > gpurun_out/phase2/${v}_s0.json 2> gpurun_out/phase2/err.txt || exit $?
  timeout -k 10 120 python -u tools/phase_group.py synthetic 2301 20000 > gpurun_out/phase2/${v}_s2301.json 2>> gpurun_out/phase2/err.txt || exit $?
  timeout -k 10 120 python -u tools/phase_group.py dmtm 500 > gpurun_out/phase2/${v}_dmtm.json 2>> gpurun_out/phase2/err.txt || exit $?
done
