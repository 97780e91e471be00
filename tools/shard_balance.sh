#!/bin/bash
# Per-rank cost of the N-GPU weak-scaling grid, emulated on one GPU (no process
# group): tools/shard_balance.sh N -> gpurun_out/shard_balance.txt
N=${1:-8}
mkdir -p gpurun_out
for sh in contiguous cyclic; do
  for r in $(seq 0 $((N - 1))); do
    timeout -k 10 120 python -u bench.py --shard $sh --emulate $r/$N --steps 3 --warmup 1 --no-cpu-baseline \
        > gpurun_out/sb.log 2>&1 || exit $?
    echo "$sh $r/$N $(tail -1 gpurun_out/sb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline"]["lane_efficiency"])')" >> gpurun_out/shard_balance.txt
  done
done
