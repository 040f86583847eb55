#!/bin/bash
# smoke() and the multi-rank bench path rehearsed on a one-GPU box: two ranks over gloo on
# GPU 0 (--same-device; not a scaling point).  gpurun_out/s8/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/s8
mkdir -p $O
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --backend gloo --same-device --collective torch --no-cpu \
  --steps 20 --warmup 5 > $O/rehearsal_2ranks.json 2> $O/rehearsal.err
