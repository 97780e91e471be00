#!/bin/bash
# Build A/B variants of the library (run HERE on the CPU host):
#   tools/ab_build.sh name1 "-DFLAG=.." name2 "-DFLAG=.." ...
# -> pycatkin_amd/_abt/lib_<name>.so (travels to the GPU box; remove after the A/B) ; run one with PCK_LIB=<path> python bench.py ...
# Variants build one after the other, each with the product's parallel split
# build (__graft_entry__.compile_library); diagnostic builds whose __device__
# counters the C-ABI reads back (-DPCK_PHASE, -DPCK_TRACE, -DPCK_WAVE_TIMES) are one
# translation unit, as the counters must live in the unit that reads them.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/pycatkin_amd/_abt"
# the hipRTC kernels compile from the embedded headers: refresh them first
(cd "$ROOT" && python3 -c "import __graft_entry__ as g; g.embed_rtc_sources()")
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  case "$flags" in
    *PCK_PHASE*|*PCK_TRACE*|*PCK_WAVE_TIMES*)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-signed-zeros -mllvm -amdgpu-sched-strategy=max-ilp \
          -shared -fPIC $flags -I"$ROOT/include" -o "$ROOT/pycatkin_amd/_abt/lib_$name.so" \
          "$ROOT/pycatkin_amd/csrc/mk_kernels.hip" -lhiprtc ;;
    *)
      (cd "$ROOT" && python3 -c "import sys, __graft_entry__ as g; g.compile_library(sys.argv[1], sys.argv[2].split())" \
          "$ROOT/pycatkin_amd/_abt/lib_$name.so" "$flags") ;;
  esac
done
ls -la "$ROOT/pycatkin_amd/_abt"
