#!/bin/bash
# one thread per tile boundary in the fix-up (16-B record loads) against one per (boundary,
# field): parity tests, then in ONE process over the SAME arrays (ref = new build)
set -euo pipefail
O=gpurun_out/r04/inproc3; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_multirank.py tests/test_gpu_fp32.py tests/test_gpu_config34.py tests/test_gpu_pipeline.py tests/test_gpu_exchange_ranks.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
export FCX_LIBRARY=ab/gfix3/libfcx.so
timeout -k 10 400 python3 $B/inproc_ab.py --group --types 2 --rounds 8 --steps 20 --warmup 40 --lib old=ab/gfix2/libfcx.so --opts nohead:98=1 > $O/t2.json
timeout -k 10 400 python3 $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 --opts nohalo:atmos_halo=0 --lib old_nohalo=ab/gfix2/libfcx.so@atmos_halo=0 --opts nohalo_nohead:atmos_halo=0,98=1 > $O/t1.json
timeout -k 10 400 python3 $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 --opts nohalo:atmos_halo=0 --lib old_nohalo=ab/gfix2/libfcx.so@atmos_halo=0 > $O/f32.json
