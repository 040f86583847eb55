#!/bin/bash
# Round evidence on a 1-GPU MI355X box, from the repo root: the default bench line, the
# rocprof kernel statistics of the same command, the PMC traffic passes (FETCH_SIZE and
# WRITE_SIZE in separate runs) and the other bench lines.  Output under gpurun_out/ev/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/ev
mkdir -p $O
B="python3 bench.py"
timeout -k 10 300 $B > $O/bench_n1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu > $O/bench_under_rocprof.json
for c in FETCH_SIZE WRITE_SIZE; do
  d=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_t1/$d -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_t2/$d -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --types 2 > /dev/null
done
timeout -k 10 300 $B --no-cpu --types 2 > $O/bench_n1_T2.json
timeout -k 10 300 $B --no-cpu --bias > $O/bench_n1_bias_config5.json
timeout -k 10 300 $B --no-cpu --precision f32 > $O/bench_n1_f32.json
echo done > $O/DONE
