#!/bin/bash
# fp32 segments summed by ordinal (contiguous atmosphere stores per round): parity of the
# fp32 and group paths, then in ONE process over the same arrays against the previous build
set -euo pipefail
O=gpurun_out/r05/ord; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_group.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
export FCX_LIBRARY=ab/ref/libfcx.so
timeout -k 10 400 python3 -u $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 \
  --lib ord=ab/ord/libfcx.so --lib ordx32=ab/ordx32/libfcx.so --lib x32=ab/f32x32/libfcx.so > $O/f32.json
