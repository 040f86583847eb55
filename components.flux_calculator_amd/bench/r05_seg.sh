#!/bin/bash
# the compacted exchange -> atmosphere map (start bits + segment cells instead of a 4-B index
# per cell): the parity of every fused path, then in ONE process over the same arrays
# against the build before it, T = 1 fp64, fp32 and T = 2
set -euo pipefail
O=gpurun_out/r05/seg; mkdir -p $O
B=components.flux_calculator_amd/bench
export FCX_LIBRARY=ab/ref5/libfcx.so
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 --lib seg=ab/seg/libfcx.so > $O/t1.json
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 --lib seg=ab/seg/libfcx.so > $O/f32.json
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --types 2 --rounds 6 --steps 20 --warmup 40 --lib seg=ab/seg/libfcx.so > $O/t2.json
