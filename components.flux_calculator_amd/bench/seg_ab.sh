#!/bin/bash
# Segment sums in rounds (product) vs the per-position loop (abx/seg0): the fused-accumulation
# tests, then fp64/fp32 x random/periodic and T = 2 random, interleaved.  gpurun_out/seg_ab/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/seg_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_fp32.py tests/test_gpu_config34.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  for cfg in "f64 random 1" "f64 periodic 1" "f32 random 1" "f64 random 2"; do
    set -- $cfg
    for lib in main seg0; do
      L=components.flux_calculator_amd/lib/libfcx.so
      [ "$lib" = main ] || L=abx/$lib/libfcx.so
      FCX_LIBRARY=$L timeout -k 10 200 python3 bench.py --no-cpu --config4 0 --other-map 0 --steps 100 --precision $1 --atmos-map $2 --types $3 > $O/${1}_${2}_T$3_${lib}_r$r.json
    done
  done
done
