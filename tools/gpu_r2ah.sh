set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile.sh r2ah/prof_ch4 python3 bench.py --config ch4 --steps 1 --warmup 1 --no-cpu-baseline || exit $?
bash tools/profile.sh r2ah/prof_dmtm python3 bench.py --config dmtm_drc --steps 1 --warmup 1 --no-cpu-baseline || exit $?
bash tools/profile.sh r2ah/prof_synthetic python3 bench.py --config synthetic --n 16384 --steps 1 --warmup 1 --no-cpu-baseline || exit $?
