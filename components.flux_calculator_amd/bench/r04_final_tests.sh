#!/bin/bash
# the round's final tree: the GPU suite as the driver runs it, and smoke()
set -euo pipefail
O=gpurun_out/r04/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
