#!/bin/bash
# the members' fix-ups as one launch against one per member (A/B build knob 99), one process
set -euo pipefail
O=gpurun_out/r04/arm4; mkdir -p $O
B=components.flux_calculator_amd/bench
export FCX_LIBRARY=ab/gfix/libfcx.so
timeout -k 10 300 python3 $B/arm_ab.py --types 2 --arms "group_fixup:random;fixup_each:random:99=1" --rounds 10 > $O/t2.json
timeout -k 10 300 python3 $B/arm_ab.py --arms "group_fixup:random:atmos_halo=0;fixup_each:random:atmos_halo=0,99=1;halo:random" --rounds 10 > $O/t1.json
timeout -k 10 300 python3 $B/arm_ab.py --precision f32 --arms "group_fixup:random:atmos_halo=0;fixup_each:random:atmos_halo=0,99=1;halo:random" --rounds 10 > $O/f32.json
