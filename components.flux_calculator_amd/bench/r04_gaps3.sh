#!/bin/bash
set -euo pipefail
O=gpurun_out/r04/gaps3; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fp32.py -k "lengths5" -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
