#!/bin/bash
# round 6: the zero-copy / host-memory test file alone (after adding the allocator layout test).
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/zc}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_zero_copy.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/test.log 2>&1; rc=$?
echo "zc rc=$rc" | tee $O/steps.txt
exit $rc
