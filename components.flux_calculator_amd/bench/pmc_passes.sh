#!/bin/bash
# PMC traffic passes of the bench kernels (MI355X_MICROARCH.md HBM section): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 runs, T = 1 and T = 2, under gpurun_out/$1.
# Then, in the build container: python components.flux_calculator_amd/bench/pmc_traffic.py
#   gpurun_out/$1/t1 --source profiles/<round>/pmc_t1  (and t2 with --types 2)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc}
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  d=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/t1/$d -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --config4 0 > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/t2/$d -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --config4 0 --types 2 > /dev/null
done
echo done > $O/DONE
