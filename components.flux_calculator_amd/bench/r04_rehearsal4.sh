#!/bin/bash
# bench.py's N > 1 path with FOUR ranks on GPU 0 through libfcx's own exchange (the mock
# librccl stand-in: RCCL refuses several ranks on one device), interior ranks with a left and
# a right boundary slot; the line's multi_gpu_check compares the shared cells with the
# sequential sum over the neighbours' exchange cells
set -euo pipefail
O=gpurun_out/r04/rehearsal4; mkdir -p $O
FCX_RCCL_LIBRARY=$PWD/components.flux_calculator_amd/lib/test/libmock_rccl.so FCX_MOCK_RCCL_LOG=$PWD/$O/calls \
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29544 bench.py --gpus 4 --backend gloo --same-device --collective rccl --steps 10 --warmup 5 \
  --no-cpu --e2e 0 --other-map 0 --config4 0 > $O/bench_rehearsal_4ranks.json 2> $O/rehearsal.err
