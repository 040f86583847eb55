#!/bin/bash
# HBM request bytes (pmc_bytes.sh: read-request sizes, then WRITE_SIZE; separate runs) of the
# fp64 T = 1 group launch after the halo launches took the compacted map
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/pmc2; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu --e2e 0 --other-map 0 --config4 0"
bash components.flux_calculator_amd/bench/pmc_bytes.sh $O/pmc_t1 -- python3 bench.py $A
echo done > $O/DONE
