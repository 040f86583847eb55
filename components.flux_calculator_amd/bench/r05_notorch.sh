#!/bin/bash
# the Baltic-size step in a process without torch (as a Fortran host: the system HIP runtime,
# engine-owned streams) against the same in a torch process
set -euo pipefail
O=gpurun_out/r05/notorch; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 300 python3 -u $B/baltic_probe.py --no-torch --steps 300 --handover 0 --mode default: --mode dma:zero_copy=0 > $O/baltic_probe_notorch.log 2>&1
timeout -k 10 300 python3 -u $B/baltic_probe.py --steps 300 --handover 0 --mode default: --mode dma:zero_copy=0 > $O/baltic_probe_torch.log 2>&1
