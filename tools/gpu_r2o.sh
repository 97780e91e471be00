set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2o
mkdir -p $O
bash tools/ab_run.sh cur nostall nopos nonegf nocrows noall || exit $?
(cd _r1ab && timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline) > $O/r1.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dump_synth.py 65536 > $O/synth.log 2>&1 || exit $?
