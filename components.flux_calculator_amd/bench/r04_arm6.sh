#!/bin/bash
# whole-line crossing records (one wave writes each record) against HEAD's two-writer records:
# parity tests, then each build's random map against its periodic map (no records: the
# control) in one process, builds alternated; kernel times from a trace in a second pass
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/arm6; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_multirank.py tests/test_gpu_fp32.py tests/test_gpu_config34.py tests/test_gpu_pipeline.py tests/test_gpu_exchange_ranks.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  for lib in new head; do
    L=components.flux_calculator_amd/lib/libfcx.so; [ $lib = head ] && L=ab/head/libfcx.so
    FCX_LIBRARY=$L timeout -k 10 300 python3 $B/arm_ab.py --types 2 --arms "random:random;periodic:periodic" --rounds 6 > $O/t2_${lib}_r$r.json
    FCX_LIBRARY=$L timeout -k 10 300 python3 $B/arm_ab.py --arms "halo:random;nohalo:random:atmos_halo=0;periodic:periodic" --rounds 6 > $O/t1_${lib}_r$r.json
  done
done
for lib in new head; do
  L=components.flux_calculator_amd/lib/libfcx.so; [ $lib = head ] && L=ab/head/libfcx.so
  FCX_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$lib -o run -- python3 $B/arm_ab.py --types 2 --arms "random:random;periodic:periodic" --rounds 4 > $O/tr_$lib.json
  python3 $B/split_trace.py $O/tr_$lib/run_kernel_trace.csv $O/tr_$lib.json > $O/tr_${lib}_split.json
done
