#!/bin/bash
# Default bench with the periodic atmosphere map (runs never cross a wave tile) against the
# random-run map (segments cross wave tiles: carry hand-offs), interleaved; then the random
# map with contiguous caller arrays, and its rocprof kernel statistics.  gpurun_out/amap/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/amap
mkdir -p $O
for m in periodic random periodic random; do
  timeout -k 10 200 python3 bench.py --no-cpu --config4 0 --steps 100 --atmos-map $m > $O/$m.json
  mv $O/$m.json $O/${m}_$(date +%s%N).json
done
timeout -k 10 200 python3 bench.py --no-cpu --config4 0 --steps 100 --atmos-map random --caller-device > $O/random_caller.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_random -o run -- python3 bench.py --no-cpu --config4 0 --steps 50 --warmup 50 --atmos-map random > /dev/null
