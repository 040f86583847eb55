#!/bin/bash
# fp32 group kernel (config 5): launch-shape A/B in ONE process over the same arrays
# (XCD run length 16/32/64 workgroups, 4 or 8 waves per block), then the fp32 bench line
set -euo pipefail
O=gpurun_out/r05/f32ab; mkdir -p $O
B=components.flux_calculator_amd/bench
export FCX_LIBRARY=ab/ref/libfcx.so
timeout -k 10 400 python3 -u $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 \
  --lib x32=ab/f32x32/libfcx.so --lib x64=ab/f32x64/libfcx.so --lib w8=ab/f32w8/libfcx.so > $O/f32.json
unset FCX_LIBRARY
timeout -k 10 300 python3 -u bench.py --precision f32 --no-cpu --e2e 0 --other-map 0 --config4 0 > $O/bench_f32_a.json
timeout -k 10 300 python3 -u bench.py --precision f32 --bias --no-cpu --e2e 0 --other-map 0 --config4 0 > $O/bench_f32_bias.json
