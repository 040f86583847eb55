#!/bin/bash
# Round-3 profiles: request-size HBM traffic passes (bench/pmc_bytes.sh) and SQ wave-state
# counters of a short bench line.  r03_profile.sh OUTDIR NAME "BENCH ARGS" [NAME "ARGS" ...]
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
while [ $# -gt 1 ]; do
  N=$1; A=$2; shift 2
  bash components.flux_calculator_amd/bench/pmc_bytes.sh $O/pmc_$N -- python3 bench.py $A
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/sq_$N -o run \
    -- python3 bench.py $A > /dev/null
done
