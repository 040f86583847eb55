#!/bin/bash
# where the random map's T = 2 kernel time goes: head records off (A/B knob 98, wrong
# crossing values) against the default and the periodic map, kernel times from a trace
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/arm5; mkdir -p $O
B=components.flux_calculator_amd/bench
export FCX_LIBRARY=ab/gfix/libfcx.so
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t2 -o run -- python3 $B/arm_ab.py --types 2 --arms "random:random;nohead:random:98=1;periodic:periodic" --rounds 6 > $O/t2.json
python3 $B/split_trace.py $O/t2/run_kernel_trace.csv $O/t2.json > $O/t2_split.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t1 -o run -- python3 $B/arm_ab.py --arms "nohalo:random:atmos_halo=0;nohead:random:atmos_halo=0,98=1;periodic:periodic;halo:random" --rounds 6 > $O/t1.json
python3 $B/split_trace.py $O/t1/run_kernel_trace.csv $O/t1.json > $O/t1_split.json
