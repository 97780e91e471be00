#!/bin/bash
# rocprofv3 runs of one workload: kernel trace + stats, then separate PMC
# passes (one counter block set per pass).  Outputs under gpurun_out/$1.
#   tools/profile.sh OUT                  -> the bench.py volcano workload
#   tools/profile.sh OUT python3 tools/bench_configs.py --configs ch4 --reps 1
set -u
OUT=${1:-prof}
shift
if [ $# -eq 0 ]; then set -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$OUT
run() {  # name, rocprof args... (the workload command follows --)
  local name=$1; shift
  timeout -k 10 170 rocprofv3 "$@" --output-format csv -d gpurun_out/$OUT/$name -o run -- "${CMD[@]}" \
      > gpurun_out/$OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/$OUT/summary.txt
  return $rc
}
CMD=("$@")
run trace --kernel-trace --stats || exit $?
run pmc_fetch --pmc FETCH_SIZE || exit $?
run pmc_write --pmc WRITE_SIZE || exit $?
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run pmc_f64 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU || exit $?
run pmc_f32 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVES || exit $?
exit 0
