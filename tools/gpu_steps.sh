#!/bin/bash
# One GPU-box session (run through gpurun): the named steps in order, each
# under its own time limit, outputs under gpurun_out/$OUT; the session stops
# at the first step that fails (a GPU fault, abort, segfault or time limit
# ends everything after it).
#
#   tools/gpu_steps.sh OUT STEP [STEP ...]
#
#   tests              pytest -m gpu (whole suite)           -> OUT/tests.log
#   tests:EXPR         pytest -m gpu -k EXPR (, = space)     -> OUT/tests.log (appended)
#   testsall[:EXPR]    the same without -x (every failure)   -> OUT/tests.log (appended)
#   smoke              __graft_entry__.smoke()               -> OUT/smoke.log
#   bench:ARGS         python bench.py ARGS (',' = ' ')      -> OUT/bench_<n>.json / .err
#   benchlong:ARGS     the same with a 1000 s limit (synthetic 1e6)
#   abbench:NAME:ARGS  bench.py ARGS on the A/B build pycatkin_amd/_abt/lib_NAME.so
#   envbench:V=X:ARGS  bench.py ARGS with the environment variable V=X
#   abenv:NAME:V=X:ARGS  abbench with the environment variable V=X
#   py:SCRIPT,ARGS     python SCRIPT ARGS                    -> OUT/py_<n>.log
#   profile:NAME:ARGS  tools/profile.sh OUT/NAME python3 bench.py ARGS
#   ab:NAME,NAME...    tools/ab_run.sh variants (pycatkin_amd/_abt/lib_NAME.so)
set -u
OUT=$1
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/$OUT
k=0
for step in "$@"; do
  k=$((k + 1))
  kind=${step%%:*}
  arg=""
  [ "$kind" != "$step" ] && arg=${step#*:}
  echo "[gpu_steps] $(date +%T) step $k: $step" | tee -a gpurun_out/$OUT/steps.log
  case $kind in
    tests|testsall)
      if [ -n "$arg" ]; then sel=(-k "${arg//,/ }"); else sel=(); fi
      if [ "$kind" = tests ]; then sel+=(-x); fi
      timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA --timeout 160 --timeout-method thread "${sel[@]}" \
          >> gpurun_out/$OUT/tests.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 ;;
    bench)
      timeout -k 10 400 python -u bench.py ${arg//,/ } > gpurun_out/$OUT/bench_$k.json 2> gpurun_out/$OUT/bench_$k.err ;;
    abbench)            # abbench:NAME:ARGS -- bench.py ARGS on pycatkin_amd/_abt/lib_NAME.so
      name=${arg%%:*}
      bargs=${arg#*:}
      PCK_LIB=$PWD/pycatkin_amd/_abt/lib_$name.so timeout -k 10 400 python -u bench.py ${bargs//,/ } \
          > gpurun_out/$OUT/bench_$k.json 2> gpurun_out/$OUT/bench_$k.err ;;
    envbench)           # envbench:VAR=VALUE:ARGS -- bench.py ARGS with one environment variable set
      kv=${arg%%:*}
      bargs=${arg#*:}
      env "$kv" timeout -k 10 400 python -u bench.py ${bargs//,/ } \
          > gpurun_out/$OUT/bench_$k.json 2> gpurun_out/$OUT/bench_$k.err ;;
    abenv)              # abenv:NAME:VAR=VALUE:ARGS -- abbench with one environment variable set
      name=${arg%%:*}
      rest=${arg#*:}
      kv=${rest%%:*}
      bargs=${rest#*:}
      env "$kv" PCK_LIB=$PWD/pycatkin_amd/_abt/lib_$name.so timeout -k 10 400 python -u bench.py ${bargs//,/ } \
          > gpurun_out/$OUT/bench_$k.json 2> gpurun_out/$OUT/bench_$k.err ;;
    benchlong)
      timeout -k 10 1000 python -u bench.py ${arg//,/ } > gpurun_out/$OUT/bench_$k.json 2> gpurun_out/$OUT/bench_$k.err ;;
    pyin)              # pyin:DIR:ARGS -- python ARGS run inside DIR
      d=${arg%%:*}; pargs=${arg#*:}
      (cd $d && timeout -k 10 400 python -u ${pargs//,/ }) > gpurun_out/$OUT/py_$k.log 2>&1 ;;
    py)
      timeout -k 10 400 python -u ${arg//,/ } > gpurun_out/$OUT/py_$k.log 2>&1 ;;
    profile)
      name=${arg%%:*}
      bargs=${arg#*:}
      bash tools/profile.sh $OUT/$name python3 bench.py ${bargs//,/ } ;;
    ab)
      bash tools/ab_run.sh ${arg//,/ } ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "[gpu_steps] $(date +%T) step $k rc=$rc" | tee -a gpurun_out/$OUT/steps.log
  # failed tests (pytest rc 1) or a script's own assertion (python rc 1) do not
  # end the session; anything else (fault, abort, segfault, time limit) does
  if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && { [ "$kind" = tests ] || [ "$kind" = testsall ] || [ "$kind" = py ]; }; }; then exit $rc; fi
done
exit 0
