#!/bin/bash
# Event-pair cost in the timed steps: bench.py with one pair per step (around the dominant
# engine, the default) against a pair around every engine, interleaved on one box.
# Output under gpurun_out/$1.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-events_ab}
mkdir -p $O
for r in 1 2; do
  for m in all dominant; do
    timeout -k 10 200 python3 bench.py --steps 200 --warmup 200 --no-cpu --e2e 0 --other-map 0 --config4 0 \
      --kernel-events $m > $O/bench_${m}_$r.json || exit $?
  done
done
