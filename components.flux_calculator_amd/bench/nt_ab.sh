#!/bin/bash
# Atmosphere-output stores: plain (product) vs non-temporal (abx/nt1: all; abx/nt2: the lines
# a tile owns whole), fp64 random / periodic and fp32 random, interleaved.  gpurun_out/nt_ab/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/nt_ab
mkdir -p $O
for r in 1 2; do
  for cfg in "f64 random" "f64 periodic" "f32 random"; do
    set -- $cfg
    for lib in main nt1 nt2; do
      L=components.flux_calculator_amd/lib/libfcx.so
      [ "$lib" = main ] || L=abx/$lib/libfcx.so
      FCX_LIBRARY=$L timeout -k 10 200 python3 bench.py --no-cpu --config4 0 --other-map 0 --steps 100 --precision $1 --atmos-map $2 > $O/${1}_${2}_${lib}_r$r.json
    done
  done
done
