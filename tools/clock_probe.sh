#!/bin/bash
# Sample the GPU's shader clock and power while bench.py runs one condition order:
#   tools/clock_probe.sh row|tile  -> gpurun_out/clock_<order>.txt
o=$1
mkdir -p gpurun_out
( for i in $(seq 1 60); do rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|Power \(" | tr '\n' ' '; echo; sleep 0.5; done ) > gpurun_out/clock_$o.txt &
sp=$!
timeout -k 10 120 python -u bench.py --order $o --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/clk_bench_$o.log 2>&1
rc=$?
kill $sp 2>/dev/null
exit $rc
