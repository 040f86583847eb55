#!/bin/bash
# round 6: D2H rate by host-allocation flags (d2h_flags_probe), the T = 2 occupancy A/B
# (next-type prefetch off / 4 waves per SIMD, in one process over the same arrays), then the
# whole GPU suite
set -euo pipefail
O=${1:-gpurun_out/r06/second}; mkdir -p $O
timeout -k 10 200 components.flux_calculator_amd/lib/probe/d2h_flags_probe 200 > $O/d2h_flags.json
cat $O/d2h_flags.json
timeout -k 10 300 python3 -u components.flux_calculator_amd/bench/inproc_ab.py --types 2 --group --rounds 8 --steps 20 \
  --lib nopf=ab/t2nopf/libfcx.so --lib nopf4=ab/t2nopf4/libfcx.so --lib pf4=ab/t2pf4/libfcx.so > $O/t2_ab.json 2> $O/t2_ab.err
tail -c 1500 $O/t2_ab.json
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests \
  > $O/tests.log 2>&1
tail -5 $O/tests.log
