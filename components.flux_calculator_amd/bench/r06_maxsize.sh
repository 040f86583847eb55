#!/bin/bash
# round 6: the 200M-cell MOM5 test (offsets past int32 in the tiled read pool), timed.
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/maxsize}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_max_size.py -x -v -m gpu --timeout 600 --timeout-method thread \
  -p no:cacheprovider --durations=0 > $O/test.log 2>&1; rc=$?
echo "maxsize rc=$rc" | tee $O/steps.txt
exit $rc
