#!/bin/bash
# tools/ab_configs.sh CONFIGS name1 name2 ... : bench_configs on A/B library variants (GPU box)
mkdir -p gpurun_out/ab
cfg=$1; shift
for name in "$@"; do
  PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_$name.so timeout -k 10 200 python tools/bench_configs.py --configs $cfg \
      --reps 2 > gpurun_out/ab/cfg_$name.log 2>&1 || exit $?
  grep solves_per_s gpurun_out/ab/cfg_$name.log | python -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print("'$name'", d["config"], d["seconds_per_launch"], d["solves_per_s"], d["status"])' >> gpurun_out/ab/cfg_summary.txt
done
