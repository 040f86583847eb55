#!/bin/bash
# Crossing records (product) vs separate carry / head / head-product arrays (abx/prev): the
# fused-accumulation tests, then fp64 random, fp32 random, T = 2 random, interleaved, and
# rocprof statistics of both on fp64 random.  gpurun_out/xrec_ab/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/xrec_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_fp32.py tests/test_gpu_config34.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  for cfg in "f64 1" "f32 1" "f64 2"; do
    set -- $cfg
    for lib in main prev; do
      L=components.flux_calculator_amd/lib/libfcx.so
      [ "$lib" = main ] || L=abx/$lib/libfcx.so
      FCX_LIBRARY=$L timeout -k 10 200 python3 bench.py --no-cpu --config4 0 --other-map 0 --steps 100 --precision $1 --types $2 > $O/${1}_T$2_${lib}_r$r.json
    done
  done
done
for lib in main prev; do
  L=components.flux_calculator_amd/lib/libfcx.so
  [ "$lib" = main ] || L=abx/$lib/libfcx.so
  FCX_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$lib -o run -- python3 bench.py --no-cpu --config4 0 --other-map 0 --steps 50 --warmup 50 > /dev/null
done
