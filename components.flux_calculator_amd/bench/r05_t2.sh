#!/bin/bash
# round 5: the new GPU tests (async phase, run_group at config-3 size, exchange scenarios),
# then the default bench line (N = 1) with the Baltic-size async drop-in and the link bound.
O=gpurun_out/r05/t2; mkdir -p $O
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step gpu_tests 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_fortran.py tests/test_gpu_config34.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
step bench 500 python -u bench.py
