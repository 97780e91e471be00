set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4l
run() { name=$1; shift; timeout -k 10 400 "$@" > gpurun_out/r4l/$name.json 2> gpurun_out/r4l/$name.err; echo "$name rc=$?" >> gpurun_out/r4l/steps.log; }
run vol_base python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
run vol_netexact env PCK_LIB=$PWD/pycatkin_amd/_abx/lib_netexact.so python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
run cstr_base python -u bench.py --config cstr --steps 5 --warmup 2 --no-cpu-baseline
run cstr_netexact env PCK_LIB=$PWD/pycatkin_amd/_abx/lib_netexact.so python -u bench.py --config cstr --steps 5 --warmup 2 --no-cpu-baseline
run drc_tables python -u bench.py --config dmtm_drc --steps 3 --warmup 1 --no-cpu-baseline
run drc_ct env PCK_GRP_CT=1 python -u bench.py --config dmtm_drc --steps 3 --warmup 1 --no-cpu-baseline
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rA --timeout 160 --timeout-method thread -k "synthetic_fixture" > gpurun_out/r4l/tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/r4l/steps.log
exit 0
