#!/bin/bash
# the compacted exchange -> atmosphere map (start bits + segment cells instead of a 4-B index
# per cell): the fused paths' parity, then in ONE process over the same arrays against the
# build before it (ref5), the dependent loads before (seg) or after (seg2) the flux pass;
# T = 1 fp64, fp32 and T = 2
set -euo pipefail
O=gpurun_out/r05/seg; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_fp32.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_config34.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
export FCX_LIBRARY=ab/ref5/libfcx.so
L="--lib seg=ab/seg/libfcx.so --lib seg2=ab/seg2/libfcx.so"
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 $L > $O/t1.json
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 $L > $O/f32.json
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --types 2 --rounds 6 --steps 20 --warmup 40 $L > $O/t2.json
