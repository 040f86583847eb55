#!/bin/bash
# group fix-up (one launch for the members' crossing records): tests, then halo tiles against
# records + the group fix-up in one process, T = 1 fp64 / fp32, and T = 2
set -euo pipefail
O=gpurun_out/r04/arm3; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_group.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 $B/arm_ab.py --arms "halo:random;nohalo:random:atmos_halo=0;periodic:periodic" --rounds 10 > $O/t1.json
timeout -k 10 300 python3 $B/arm_ab.py --precision f32 --arms "halo:random;nohalo:random:atmos_halo=0;periodic:periodic" --rounds 10 > $O/f32.json
timeout -k 10 300 python3 $B/arm_ab.py --types 2 --arms "random:random;periodic:periodic" --rounds 8 > $O/t2.json
