#!/bin/bash
# the compacted map in every fp64 launch (ab/c2: -DFCX_F64_COMPACT=2, the crossing records'
# first cell from a per-tile array) against the product build (1: halo launches only) and
# the index-only build (ab/idx): parity of both builds, then in ONE process over the same
# arrays T = 2 (records), T = 1 on the periodic map (no crossings) and T = 1 random (halo)
set -euo pipefail
O=gpurun_out/r05/f64seg2; mkdir -p $O
B=components.flux_calculator_amd/bench
T="tests/test_gpu_parity.py tests/test_gpu_group.py tests/test_gpu_config34.py tests/test_gpu_layout.py tests/test_gpu_multirank.py tests/test_gpu_driver.py"
timeout -k 10 400 python3 -u -m pytest $T tests/test_gpu_fp32.py -x -q -p no:cacheprovider > $O/tests_product.log 2>&1
FCX_LIBRARY=ab/c2/libfcx.so timeout -k 10 400 python3 -u -m pytest $T -x -q -p no:cacheprovider > $O/tests_c2.log 2>&1
L="--lib c2=ab/c2/libfcx.so --lib idx=ab/idx/libfcx.so"
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --types 2 --rounds 6 --steps 20 --warmup 40 $L > $O/t2.json
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --atmos-map periodic --rounds 8 --steps 20 --warmup 40 $L > $O/t1_periodic.json
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 $L > $O/t1.json
