#!/bin/bash
# After the fix-up rework: GPU suite, the default bench (random map, other_map sub-object)
# with the driver's arguments, and the hand-off A/B.  gpurun_out/s6/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/s6
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_w5.json
bash components.flux_calculator_amd/bench/handoff_ab.sh
