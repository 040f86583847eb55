#!/bin/bash
# the bench line's spread on ONE box: six processes one after the other, main workload only
set -euo pipefail
O=gpurun_out/r05/spread; mkdir -p $O
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python3 -u bench.py --no-cpu --e2e 0 --other-map 0 --config4 0 > $O/bench_$i.log 2>&1
done
