#!/bin/bash
# atmosphere cells without exchange cells (runs of 0..5 / 0..10): the previous build leaves
# their fused outputs unwritten (NaN in the test), the fixed one stores 0
set -uo pipefail
O=gpurun_out/r04/gaps; mkdir -p $O
FCX_LIBRARY=ab/base2/libfcx.so timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_multirank.py::test_fused_accumulation_long_segments" -k "lengths7 or lengths8" -q --timeout 120 --timeout-method thread > $O/before_fix.log 2>&1
echo "before rc=$?"
set -e
timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_multirank.py::test_fused_accumulation_long_segments" "tests/test_gpu_multirank.py::test_fused_accumulation_of_averages_long_segments" -k "lengths7 or lengths8 or lengths4" -v --timeout 120 --timeout-method thread > $O/after_fix.log 2>&1
echo "after ok"
