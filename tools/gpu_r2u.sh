set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2u
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit $?
bash tools/profile.sh r2u/prof_volcano python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $?
bash tools/profile.sh r2u/prof_ch4 python3 bench.py --config ch4 --steps 1 --warmup 1 --no-cpu-baseline || exit $?
bash tools/profile.sh r2u/prof_synthetic python3 bench.py --config synthetic --n 16384 --steps 1 --warmup 1 --no-cpu-baseline || exit $?
for c in cstr dmtm_drc ch4 synthetic; do timeout -k 10 400 python -u bench.py --config $c --steps 2 --warmup 1 > $O/cfg_$c.log 2>&1 || exit $?; done
