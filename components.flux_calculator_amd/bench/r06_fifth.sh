#!/bin/bash
# round 6: the whole GPU suite again after the fixes, the 8-rank rehearsal of bench.py's
# N > 1 path, then the T = 2 occupancy counters.  Stops at the first step that faults.
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/fifth}; mkdir -p $O
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step gpu_tests 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider
step rehearsal8 700 bash components.flux_calculator_amd/bench/r06_rehearsal8.sh gpurun_out/r06/rehearsal8
step t2counters 900 bash components.flux_calculator_amd/bench/r06_t2counters.sh gpurun_out/r06/t2counters
