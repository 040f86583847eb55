#!/bin/bash
# fp64 group launch: XCD run length 32 / 64 (current) / 128 workgroups, in ONE process over
# the same arrays; T = 1 and T = 2
set -euo pipefail
O=gpurun_out/r05/xcd64; mkdir -p $O
B=components.flux_calculator_amd/bench
export FCX_LIBRARY=ab/ref5/libfcx.so
timeout -k 10 400 python3 -u $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 \
  --lib x32=ab/x32d/libfcx.so --lib x128=ab/x128d/libfcx.so > $O/t1.json
timeout -k 10 400 python3 -u $B/inproc_ab.py --group --types 2 --rounds 6 --steps 20 --warmup 40 \
  --lib x32=ab/x32d/libfcx.so --lib x128=ab/x128d/libfcx.so > $O/t2.json
