#!/bin/bash
# Carries of segments that cross a 128-cell wave tile: atmos_fixup_kernel after the launch
# (default) vs the in-launch hand-off (--carry-handoff 1), on the periodic map (no segment
# crosses a tile: no fix-up launch) and the random-run map (most tiles carry), interleaved;
# then rocprof kernel statistics of the default on the random map.  gpurun_out/handoff/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/handoff
mkdir -p $O
for r in 1 2; do
  for m in random periodic; do
    timeout -k 10 200 python3 bench.py --no-cpu --config4 0 --steps 100 --atmos-map $m > $O/${m}_fixup_r$r.json
    timeout -k 10 200 python3 bench.py --no-cpu --config4 0 --steps 100 --atmos-map $m --carry-handoff 1 > $O/${m}_handoff_r$r.json
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_random -o run -- python3 bench.py --no-cpu --config4 0 --steps 50 --warmup 50 --atmos-map random > /dev/null
