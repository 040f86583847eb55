#!/bin/bash
# round 6 ("price it against halo tiles again"): halo tiles at T = 2 in the
# group launch (A/B build FCX_HALO_RAVG=1) against crossing records + the group fix-up, at
# the round-6 code: parity tests on the halo build, then one process over the same arrays.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/halot2; mkdir -p $O
B=components.flux_calculator_amd/bench
FCX_LIBRARY=$PWD/ab_t2/halo/libfcx.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_multirank.py \
  -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
export FCX_LIBRARY=$PWD/ab_t2/base/libfcx.so
timeout -k 10 400 python3 $B/inproc_ab.py --group --types 2 --rounds 10 --steps 20 --warmup 40 \
  --lib halo=$PWD/ab_t2/halo/libfcx.so > $O/t2.json
