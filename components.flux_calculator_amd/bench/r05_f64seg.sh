#!/bin/bash
# the compacted exchange -> atmosphere map for the fp64 halo launches (T = 1 bench step): the
# fused paths' parity, then in ONE process over the same arrays against the index-per-cell
# build (ab/idx: -DFCX_F64_COMPACT=0), twice
set -euo pipefail
O=gpurun_out/r05/f64seg; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py tests/test_gpu_config34.py tests/test_gpu_layout.py tests/test_gpu_multirank.py -x -q -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --rounds 10 --steps 20 --warmup 40 --lib idx=ab/idx/libfcx.so > $O/t1_a.json
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --rounds 10 --steps 20 --warmup 40 --lib idx=ab/idx/libfcx.so > $O/t1_b.json
