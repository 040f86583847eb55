#!/bin/bash
# Remap A/B: library builds (LIBS: directories under abx/ holding libfcx.so; "main" = the
# product build) x interleaved rounds of bench/remap_bench.py.  Output gpurun_out/remap_ab/.
set -euo pipefail
O=gpurun_out/remap_ab
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS:-main}; do
    L=components.flux_calculator_amd/lib/libfcx.so
    [ "$lib" = main ] || L=abx/$lib/libfcx.so
    FCX_LIBRARY=$L timeout -k 10 200 python3 components.flux_calculator_amd/bench/remap_bench.py --rounds 5 ${EXTRA:-} > $O/${lib}_r$r.json
  done
done
