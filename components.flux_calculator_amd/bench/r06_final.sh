#!/bin/bash
# round 6, last check of the final tree: bench.py with its defaults (N = 1), then a rocprofv3
# kernel trace of a short bench command.
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/final}; mkdir -p $O
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step bench 600 python3 bench.py
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --e2e 0
