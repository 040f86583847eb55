#!/bin/bash
set -euo pipefail
O=gpurun_out/r04/graph; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_group.py -k "graph" -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
