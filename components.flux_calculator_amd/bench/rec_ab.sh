#!/bin/bash
# Remap records A/B (row f3): product build vs A/B builds under abx/ (LIBS), on the shuffled
# 2-link map, without (gpurun_out/remap_ab/) and with (gpurun_out/remap_ab_atm/) the fused
# atmosphere accumulation in the same step.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rec gpurun_out/remap_ab_atm
timeout -k 10 300 python -u -m pytest tests/test_gpu_remap.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rec/tests.log 2>&1
LIBS="${LIBS:-main}" EXTRA="--pack 2 --links 2" bash components.flux_calculator_amd/bench/remap_ab.sh
for r in 1 2; do
  for lib in ${LIBS:-main}; do
    L=components.flux_calculator_amd/lib/libfcx.so
    [ "$lib" = main ] || L=abx/$lib/libfcx.so
    FCX_LIBRARY=$L timeout -k 10 200 python3 components.flux_calculator_amd/bench/remap_bench.py --rounds 5 --pack 2 --links 2 --atmos > gpurun_out/remap_ab_atm/${lib}_r$r.json
  done
done
