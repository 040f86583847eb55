#!/bin/bash
# host <-> device copies with hipMemcpyDefault (the DMA probe: explicit device-to-host kinds
# into hipHostMalloc memory are slow): the staging / host-array tests, the Baltic-size probe
# and the default bench line (e2e at 10M cells and the Baltic block)
set -euo pipefail
O=gpurun_out/r05/dmakind; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_zero_copy.py tests/test_fortran.py tests/test_gpu_remap.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python3 -u $B/baltic_probe.py --steps 300 --mode default: --mode dma_seq:zero_copy=0 > $O/baltic_probe.log 2>&1
timeout -k 10 400 python3 -u bench.py > $O/bench_n1.log 2>&1
