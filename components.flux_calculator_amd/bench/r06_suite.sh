#!/bin/bash
# round 6: the whole GPU suite as the driver runs it (-x -q -m gpu) on the final tree, after
# the two files fixed last (zero-copy span runs, fp32 perturbations) on their own.
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/suite}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_zero_copy.py tests/test_gpu_fp32.py -x -q -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/fixed_files.log 2>&1; rc=$?
echo "fixed_files rc=$rc" | tee $O/steps.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu_tests rc=$rc" | tee -a $O/steps.txt
exit $rc
