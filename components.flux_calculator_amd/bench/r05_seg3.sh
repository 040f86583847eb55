#!/bin/bash
# the compacted map for fp32 engines only (fp64 keeps the 4-B index): the whole GPU suite,
# then in ONE process over the same arrays against the build before the compaction (ref5)
set -euo pipefail
O=gpurun_out/r05/seg3; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
export FCX_LIBRARY=ab/ref5/libfcx.so
L="--lib seg3=ab/seg3/libfcx.so --lib seg2=ab/seg2/libfcx.so"
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 $L > $O/f32.json
timeout -k 10 300 python3 -u $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 $L > $O/t1.json
