#!/bin/bash
# edge-line merge: parity tests, then in ONE process over the SAME arrays: merge on (ref),
# merge off (FCX_OPT_ATMOS_MERGE 0, same build) and the previous build (gfix2)
set -euo pipefail
O=gpurun_out/r04/merge1; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_multirank.py tests/test_gpu_fp32.py tests/test_gpu_config34.py tests/test_gpu_pipeline.py tests/test_gpu_exchange_ranks.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
export FCX_LIBRARY=ab/merge1/libfcx.so
timeout -k 10 400 python3 $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 --opts nomerge:atmos_merge=0 --lib old=ab/gfix2/libfcx.so > $O/t1.json
timeout -k 10 400 python3 $B/inproc_ab.py --group --types 2 --rounds 8 --steps 20 --warmup 40 --opts nomerge:atmos_merge=0 --lib old=ab/gfix2/libfcx.so > $O/t2.json
timeout -k 10 400 python3 $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 --opts nomerge:atmos_merge=0 --lib old=ab/gfix2/libfcx.so > $O/f32.json
