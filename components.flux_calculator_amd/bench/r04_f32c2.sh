#!/bin/bash
# fp32 fused kernels with 2 cells per lane (A/B build FCX_F32_CPL=2: 8-B lanes, 128-cell
# tiles, 79-88 VGPRs, 5-7 waves per SIMD) against 4 (128 VGPRs, 4 waves): the fp32 parity
# tests on the C = 2 build, then one process over the same arrays
set -euo pipefail
O=gpurun_out/r04/f32c2; mkdir -p $O
B=components.flux_calculator_amd/bench
FCX_LIBRARY=ab/c2/libfcx.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_group.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
export FCX_LIBRARY=ab/c4/libfcx.so
timeout -k 10 400 python3 $B/inproc_ab.py --group --precision f32 --rounds 10 --steps 20 --warmup 40 --lib c2=ab/c2/libfcx.so > $O/group.json
timeout -k 10 400 python3 $B/inproc_ab.py --precision f32 --rounds 8 --steps 20 --warmup 40 --lib c2=ab/c2/libfcx.so > $O/per_engine.json
