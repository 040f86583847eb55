#!/bin/bash
# the exchange with one cross-stream edge per stream and the finishes in one launch: the
# exchange-rank scenarios, then sequential against overlapped (one-rank RCCL) with a trace
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/ovprobe2; mkdir -p $O
P=components.flux_calculator_amd/bench/overlap_probe.py
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_exchange_ranks.py tests/test_gpu_multirank.py tests/test_gpu_comm.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 200 python3 -u $P > $O/probe.json 2> $O/probe.err
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $P --rounds 2 --steps 20 > $O/probe_traced.json 2> $O/trace.err
