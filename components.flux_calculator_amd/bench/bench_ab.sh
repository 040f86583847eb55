#!/bin/bash
# bench.py A/B over library builds: LIBS (directories under abx/ holding libfcx.so; "main" =
# the product build) x ROUNDS interleaved rounds, EXTRA bench arguments; then, with STATS=1,
# rocprof kernel statistics of each build.  Output gpurun_out/bench_ab/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/bench_ab
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS:-main}; do
    L=components.flux_calculator_amd/lib/libfcx.so
    [ "$lib" = main ] || L=abx/$lib/libfcx.so
    FCX_LIBRARY=$L timeout -k 10 200 python3 bench.py --no-cpu --config4 0 --other-map 0 --steps 100 ${EXTRA:-} > $O/${lib}_r$r.json
  done
done
if [ "${STATS:-0}" = 1 ]; then
  for lib in ${LIBS:-main}; do
    L=components.flux_calculator_amd/lib/libfcx.so
    [ "$lib" = main ] || L=abx/$lib/libfcx.so
    FCX_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$lib -o run -- python3 bench.py --no-cpu --config4 0 --other-map 0 --steps 50 --warmup 50 ${EXTRA:-} > /dev/null
  done
fi
