#!/bin/bash
# round 5 evidence on one MI355X box with the round's kernels: the whole GPU suite, the
# default bench line, the rocprof kernel statistics of the same command (--no-cpu), and the
# other workloads' lines.  Stops at the first step that faults or times out.
export TMPDIR=/tmp
O=${1:-gpurun_out/r05/ev}; mkdir -p $O
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step gpu_tests 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_n1 400 python3 -u bench.py
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu --e2e 0
step bench_f32 200 python3 -u bench.py --no-cpu --e2e 0 --precision f32
step bench_f32_bias 200 python3 -u bench.py --no-cpu --e2e 0 --precision f32 --bias
step bench_t2 200 python3 -u bench.py --no-cpu --e2e 0 --types 2 --other-map 0 --config4 0
step bench_bias 200 python3 -u bench.py --no-cpu --e2e 0 --bias --other-map 0 --config4 0
