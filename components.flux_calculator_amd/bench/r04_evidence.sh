#!/bin/bash
# Round-4 evidence of one build: GPU suite, smoke, the default bench line with the driver's
# arguments (CPU legs at 32,768 and 10M cells included), the T = 2 / fp32 / bias lines, the
# two-rank rehearsal of bench.py's N > 1 path through libfcx's own exchange (mock RCCL,
# both ranks on GPU 0), and config 2's latency table.  Output under gpurun_out/$1.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_evidence}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
t0=$(date +%s.%N)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_w5.json || exit $?
python3 -c "print(round($(date +%s.%N) - $t0, 1))" > $O/bench_w5_wall_s.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --e2e 0 --types 2 > $O/bench_T2.json || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --e2e 0 --precision f32 > $O/bench_f32.json || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --e2e 0 --bias > $O/bench_bias.json || exit $?
FCX_RCCL_LIBRARY=$PWD/components.flux_calculator_amd/lib/test/libmock_rccl.so FCX_MOCK_RCCL_LOG=$PWD/$O/rehearsal_calls \
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 2 --backend gloo --same-device --collective rccl --steps 10 --warmup 5 \
  --no-cpu --e2e 0 --other-map 0 --config4 0 > $O/bench_rehearsal_2ranks_libfcx_exchange.json 2> $O/rehearsal.err || exit $?
timeout -k 10 300 python3 components.flux_calculator_amd/bench/latency.py --steps 1000 > $O/latency_config2.json || exit $?
exit $rc
