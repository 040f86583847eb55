#!/bin/bash
# where the group kernel's time goes (measurement builds with wrong results, in ONE process
# over the same arrays): no atmosphere-output stores, no LDS products, trivial math; and the
# XCD run length 32 for the fp32 kernel -- fp32 and fp64
set -euo pipefail
O=gpurun_out/r05/headroom; mkdir -p $O
B=components.flux_calculator_amd/bench
export FCX_LIBRARY=ab/ref/libfcx.so
L="--lib nostore=ab/nostore/libfcx.so --lib nolds=ab/nolds/libfcx.so --lib triv=ab/triv/libfcx.so"
timeout -k 10 400 python3 -u $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 $L --lib x32=ab/f32x32/libfcx.so > $O/f32.json
timeout -k 10 400 python3 -u $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 $L > $O/f64.json
