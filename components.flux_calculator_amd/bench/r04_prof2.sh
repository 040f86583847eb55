#!/bin/bash
# the final build: the grouped gap-map test, then kernel-trace statistics of the default
# bench line (the driver's arguments) -> gpurun_out/r04/prof2
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/prof2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_group.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_under_rocprof.json
