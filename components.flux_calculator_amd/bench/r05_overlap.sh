#!/bin/bash
# the overlapped boundary exchange: the exchange-rank scenarios (mock RCCL), the group and
# parity tests, then the 4-rank rehearsal of bench.py's N > 1 path (now fcx_run_group_exchange)
O=gpurun_out/r05/overlap; mkdir -p $O
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 500 python -u -m pytest tests/test_gpu_exchange_ranks.py tests/test_gpu_group.py tests/test_gpu_config34.py -v --timeout 300 --timeout-method thread -p no:cacheprovider
step rehearsal4 420 bash components.flux_calculator_amd/bench/r05_rehearsal4.sh $O/rehearsal4
