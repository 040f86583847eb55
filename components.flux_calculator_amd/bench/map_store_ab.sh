#!/bin/bash
# Does the random map cost the fused kernels through their atmosphere-output stores?  The
# product build against a measurement build without them (FCX_DBG_ATM_NOSTORE=1, wrong
# atmosphere values), fp64 and fp32, random and periodic maps.  gpurun_out/map_store_ab/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/map_store_ab
mkdir -p $O
for p in f64 f32; do
  for m in random periodic; do
    for lib in main nostore; do
      L=components.flux_calculator_amd/lib/libfcx.so
      [ "$lib" = main ] || L=abx/$lib/libfcx.so
      FCX_LIBRARY=$L timeout -k 10 200 python3 bench.py --no-cpu --config4 0 --other-map 0 --steps 100 --precision $p --atmos-map $m > $O/${p}_${m}_$lib.json
    done
  done
done
