#!/bin/bash
# halo tiles at T = 2 in the group launch (A/B build FCX_HALO_RAVG=1) against crossing
# records + the group fix-up: parity tests on the halo build, then one process, same arrays
set -euo pipefail
O=gpurun_out/r04/halot2; mkdir -p $O
B=components.flux_calculator_amd/bench
FCX_LIBRARY=ab/halot2/libfcx.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
export FCX_LIBRARY=ab/base2/libfcx.so
timeout -k 10 400 python3 $B/inproc_ab.py --group --types 2 --rounds 10 --steps 20 --warmup 40 --lib halo=ab/halot2/libfcx.so > $O/t2.json
timeout -k 10 400 python3 $B/inproc_ab.py --group --types 3 --rounds 6 --steps 10 --warmup 20 --lib halo=ab/halot2/libfcx.so > $O/t3.json
