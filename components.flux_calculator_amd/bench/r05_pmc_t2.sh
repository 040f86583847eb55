#!/bin/bash
# HBM request bytes of the T = 2 group launch and its fix-up with the round-5 kernels
# (pmc_bytes.sh: read-request sizes, then WRITE_SIZE; separate runs)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/pmc_t2; mkdir -p $O
bash components.flux_calculator_amd/bench/pmc_bytes.sh $O/pmc_t2 -- python3 bench.py --steps 20 --warmup 5 --no-cpu --e2e 0 --other-map 0 --config4 0 --types 2
echo done > $O/DONE
