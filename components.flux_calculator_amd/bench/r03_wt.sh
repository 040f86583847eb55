#!/bin/bash
# Write-through field stores A/B (in one process over the same arrays) and the kernel-trace
# statistics of the default bench line.  Output under gpurun_out/$1.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_wt}
L="--lib wt1=ab/wt1/libfcx.so --lib wt2=ab/wt2/libfcx.so --lib refB=ref"
bash components.flux_calculator_amd/bench/ab.sh ${1:-r03_wt} t1 "$L" f32 "--precision f32 $L" t2 "--types 2 $L" || exit $?
mkdir -p $O/stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_under_rocprof.json || exit $?
