set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile.sh r2aa/prof_dmtm python3 bench.py --config dmtm_drc --steps 1 --warmup 1 --no-cpu-baseline || exit $?
