#!/bin/bash
# Run GPU test selections one by one; stop on anything worse than a test failure.
mkdir -p gpurun_out
for sel in "$@"; do
  echo "=== $sel" >> gpurun_out/tests.log
  timeout -k 10 170 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 160 --timeout-method thread -k "$sel" >> gpurun_out/tests.log 2>&1
  rc=$?
  echo "=== rc=$rc" >> gpurun_out/tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
done
exit 0
