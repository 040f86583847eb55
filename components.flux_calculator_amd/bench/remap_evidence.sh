#!/bin/bash
# Row f3 evidence on a 1-GPU box, from the repo root: the remap GPU tests, the remap bench
# (gather from the arrays vs packed records, 1 and 2 links per cell, and the geometric map),
# and PMC FETCH_SIZE / WRITE_SIZE passes of the 2-link map for each gather (separate runs).
# Output under gpurun_out/remap/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/remap
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_remap.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
R="python3 components.flux_calculator_amd/bench/remap_bench.py"
timeout -k 10 300 $R > $O/remap_bench.json
timeout -k 10 300 $R --map geometric > $O/remap_bench_geometric.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $R --rounds 2 > /dev/null
for p in 0 2; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_pack$p/$c -o run -- $R --pack $p --links 2 --rounds 1 --reps 2 > /dev/null
  done
done
echo done > $O/DONE
