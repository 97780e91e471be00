set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 120 python -u tools/dump_steps.py steps_tile > $O/dump.log 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/cur_$i.log 2>&1 || exit $?
(cd _r1ab && timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline) > $O/r1_$i.log 2>&1 || exit $?
done
for c in cstr ch4 dmtm_drc synthetic; do
timeout -k 10 400 python -u bench.py --config $c --steps 2 --warmup 1 > $O/cfg_$c.log 2>&1 || exit $?
done
