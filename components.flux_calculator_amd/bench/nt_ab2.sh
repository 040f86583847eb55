#!/bin/bash
# NT fp64 atmosphere stores (product default) vs plain (abx/nt0): the full GPU suite, then
# T = 2 random, fp64 random, config 4 40M random, interleaved.  gpurun_out/nt_ab2/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/nt_ab2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for r in 1 2; do
  for cfg in "--types 2" "--types 1" "--global-cells 40000000"; do
    tag=$(echo $cfg | tr -d ' -')
    for lib in main nt0; do
      L=components.flux_calculator_amd/lib/libfcx.so
      [ "$lib" = main ] || L=abx/$lib/libfcx.so
      FCX_LIBRARY=$L timeout -k 10 300 python3 bench.py --no-cpu --config4 0 --other-map 0 --steps 50 $cfg > $O/${tag}_${lib}_r$r.json
    done
  done
done
