#!/bin/bash
# round 6: the whole GPU suite twice more without -x (every failure listed), to find tests
# whose result depends on the run (the id-reuse defect of test_span_runs_follow_the_allocation_order).
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/suite2}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 900 python3 -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests_$i.log 2>&1; rc=$?
  echo "gpu_tests_$i rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
