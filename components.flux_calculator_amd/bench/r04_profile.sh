#!/bin/bash
# Round-4 profiles: kernel-trace statistics of the default bench line (the driver's
# arguments), then request-size HBM traffic passes (bench/pmc_bytes.sh) of the T = 1, fp32
# and T = 2 workloads, whose timed launches are the group kernel.  Output under gpurun_out/$1.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_under_rocprof.json
A="--steps 20 --warmup 5 --no-cpu --e2e 0 --other-map 0 --config4 0"
for spec in "t1|$A" "f32|$A --precision f32" "t2|$A --types 2"; do
  N=${spec%%|*}; ARGS=${spec#*|}
  bash components.flux_calculator_amd/bench/pmc_bytes.sh $O/pmc_$N -- python3 bench.py $ARGS
done
