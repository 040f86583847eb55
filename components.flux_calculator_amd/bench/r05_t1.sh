#!/bin/bash
# round 5, first box: the whole GPU suite in the driver's order (no -x: every failure
# named), the host-link probe at the Baltic size, the 4-rank rehearsal of bench.py's N > 1
# path with every sub-measurement.  Stops at the first step that faults or times out.
O=gpurun_out/r05/t1; mkdir -p $O
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step rehearsal4 420 bash components.flux_calculator_amd/bench/r05_rehearsal4.sh $O/rehearsal4
step link_probe 150 python -u components.flux_calculator_amd/bench/link_probe.py --reps 300
step gpu_tests 580 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
