#!/bin/bash
# Run the bench on every A/B variant (GPU box): tools/ab_run.sh name1 name2 ...
mkdir -p gpurun_out/ab
for name in "$@"; do
  PCK_LIB=$GRAFT_REPO_ROOT/pycatkin_amd/_ab/lib_$name.so timeout -k 10 120 python bench.py --steps 5 --warmup 1 \
      --no-cpu-baseline > gpurun_out/ab/$name.log 2>&1 || exit $?
  echo "$name $(tail -1 gpurun_out/ab/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline"]["integrator_steps"], d["status"])')" >> gpurun_out/ab/summary.txt
done
