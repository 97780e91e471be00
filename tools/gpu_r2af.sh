set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2af
mkdir -p $O
for v in main prev; do
  if [ $v = main ]; then L=; else L=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_$v.so; fi
  for c in ch4 dmtm_drc; do PCK_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/${v}_$c.log 2>&1 || exit $?; done
  PCK_LIB=$L timeout -k 10 200 python -u tools/dump_synth.py 65536 > $O/${v}_synth.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py -x -v --timeout 300 --timeout-method thread > $O/gpu_group.txt 2>&1 || exit $?
