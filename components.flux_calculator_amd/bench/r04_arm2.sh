#!/bin/bash
# halo tiles against crossing records + fix-ups, grouped step, no profiler attached (a kernel
# trace inflates the short fix-up launches): T = 1 fp64 and fp32, random map, periodic beside
set -euo pipefail
O=gpurun_out/r04/arm2; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 300 python3 $B/arm_ab.py --arms "halo:random;nohalo:random:atmos_halo=0;periodic:periodic" --rounds 10 > $O/t1.json
timeout -k 10 300 python3 $B/arm_ab.py --precision f32 --arms "halo:random;nohalo:random:atmos_halo=0;periodic:periodic" --rounds 10 > $O/f32.json
timeout -k 10 300 python3 $B/arm_ab.py --arms "nohalo:random:atmos_halo=0;halo:random" --rounds 10 > $O/t1_rev.json
