#!/bin/bash
# round 6 evidence on one MI355X box with the round's code: the whole GPU suite (-x, as the
# driver runs it), smoke, the default bench line, the rocprof kernel statistics of the bench
# command (--no-cpu), the HBM request-byte passes of the timed launch, and the other
# workloads' lines.  Stops at the first step that faults or times out.
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/ev}; mkdir -p $O
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step gpu_tests 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 600 python3 -u bench.py
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu --e2e 0
step pmc 300 bash components.flux_calculator_amd/bench/pmc_bytes.sh $O/pmc_t1 -- python3 bench.py --steps 20 --warmup 5 --no-cpu --e2e 0 --other-map 0 --config4 0 --config5 0
step bench_t2 300 python3 -u bench.py --no-cpu --e2e 0 --types 2 --other-map 0 --config4 0 --config5 0
step bench_bias 300 python3 -u bench.py --no-cpu --e2e 0 --bias --other-map 0 --config4 0
step bench_f32 300 python3 -u bench.py --no-cpu --e2e 0 --precision f32 --other-map 0 --config4 0
