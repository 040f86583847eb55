#!/bin/bash
# round 6: library memory mapped non-coherently (A/B build ab_pin/nc, -DFCX_PIN_NONCOHERENT=1)
# against the same source without it (ab_pin/ref): the zero-copy tests on the NC build, then the
# Baltic-size zero-copy step alternately, one process per run (bench/libmem_ab.py).
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/pinnc}; mkdir -p $O
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
export FCX_LIBRARY=$PWD/ab_pin/nc/libfcx.so
step zc_tests_nc 400 python3 -u -m pytest tests/test_gpu_zero_copy.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do
  for b in ref nc; do
    FCX_LIBRARY=$PWD/ab_pin/$b/libfcx.so step ab_${b}_$r 200 python3 components.flux_calculator_amd/bench/libmem_ab.py --steps 500
    cat $O/ab_${b}_$r.log | grep '^{' >> $O/ab.jsonl
  done
done
