#!/bin/bash
# overlapped exchange variants (one-rank RCCL, rank 0's half of a 2-rank grid): the boundary
# tiles on the engines' stream first (ov1) or beside the main launch on the side stream
# (ov0), the all-reduce queued before the main launch in both; plus a kernel trace of ov1
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/ovprobe; mkdir -p $O
P=components.flux_calculator_amd/bench/overlap_probe.py
FCX_LIBRARY=ab/ov1/libfcx.so timeout -k 10 200 python3 -u $P > $O/ov1.json 2> $O/ov1.err
FCX_LIBRARY=ab/ov0/libfcx.so timeout -k 10 200 python3 -u $P > $O/ov0.json 2> $O/ov0.err
FCX_LIBRARY=ab/ov1/libfcx.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $P --rounds 2 --steps 20 > $O/ov1_traced.json 2> $O/trace.err
