#!/bin/bash
# round 6: span schedules on portable host memory, the Baltic-size library-memory step on both
# transports next to the link floors, then the host-memory GPU tests
set -euo pipefail
O=${1:-gpurun_out/r06/third}; mkdir -p $O
timeout -k 10 120 components.flux_calculator_amd/lib/probe/span_probe 32768 300 mapped_portable > $O/span_probe_mapped_portable.json
cat $O/span_probe_mapped_portable.json
timeout -k 10 300 python3 -u components.flux_calculator_amd/bench/libmem_probe.py > $O/libmem_probe.json 2> $O/libmem_probe.err
cat $O/libmem_probe.json
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_zero_copy.py \
  tests/test_gpu_pipeline.py tests/test_fortran.py > $O/tests.log 2>&1
tail -5 $O/tests.log
