#!/bin/bash
# Build A/B variants of the library (run HERE on the CPU host):
#   tools/ab_build.sh name1 "-DFLAG=.." name2 "-DFLAG=.." ...
# -> pycatkin_amd/_ab/lib_<name>.so ; run one with PCK_LIB=<path> python bench.py ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/pycatkin_amd/_ab"
# the hipRTC kernels compile from the embedded headers: refresh them first
(cd "$ROOT" && python3 -c "import __graft_entry__ as g; g.embed_rtc_sources()")
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-signed-zeros -mllvm -amdgpu-sched-strategy=max-ilp -shared -fPIC $flags -I"$ROOT/include" \
      -o "$ROOT/pycatkin_amd/_ab/lib_$name.so" "$ROOT/pycatkin_amd/csrc/mk_kernels.hip" -lhiprtc &
done
wait
ls -la "$ROOT/pycatkin_amd/_ab"
