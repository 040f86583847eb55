#!/bin/bash
# zero-copy Baltic step with a capped grid (grid-stride waves: a wave's next reads over the
# link overlap its previous stores) against the full grid
set -euo pipefail
O=gpurun_out/r05/zcgrid; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 300 python3 -u $B/baltic_probe.py --steps 300 --handover 0 --mode default: --mode mb8:max_blocks=8 --mode mb16:max_blocks=16 --mode mb32:max_blocks=32 --mode mb64:max_blocks=64 --mode mb128:max_blocks=128 > $O/baltic_probe.log 2>&1
