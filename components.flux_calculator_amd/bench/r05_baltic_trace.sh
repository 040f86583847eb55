#!/bin/bash
# where the Baltic-size async step (three engines, staging arena + DMA) spends its time: the
# kernel and memory-copy timeline of baltic_probe's dma_seq mode under rocprofv3, and the link
# probe with libfcx's copy kind
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/baltic_trace; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 120 python3 -u $B/link_probe.py --reps 200 > $O/link_probe.json 2> $O/link_probe.err
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 $B/baltic_probe.py --steps 100 --mode dma_seq:zero_copy=0 --handover 0 > $O/probe.log 2>&1
