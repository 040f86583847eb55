#!/bin/bash
# cost of the crossing records on the SAME engines and arrays: head records off (A/B knob 98:
# wrong crossing values), and the members' fix-ups one launch each (knob 99)
set -euo pipefail
O=gpurun_out/r04/inproc2; mkdir -p $O
B=components.flux_calculator_amd/bench
export FCX_LIBRARY=ab/gfix2/libfcx.so
timeout -k 10 400 python3 $B/inproc_ab.py --group --types 2 --rounds 8 --steps 20 --warmup 40 --opts nohead:98=1 --opts each:99=1 > $O/t2.json
timeout -k 10 400 python3 $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 --opts nohalo:atmos_halo=0 --opts nohalo_nohead:atmos_halo=0,98=1 > $O/t1.json
timeout -k 10 400 python3 $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 --opts nohalo:atmos_halo=0 --opts nohalo_nohead:atmos_halo=0,98=1 > $O/f32.json
