#!/bin/bash
# Round-3 check on one MI355X: the GPU suite, config-2 latency (host transports), the default
# bench line with the driver's arguments.  Output under gpurun_out/$1 (default r03).
# A failing test (pytest exit 1) does not stop the measurements; a hang, timeout or crash
# of any step ends the script there.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 components.flux_calculator_amd/bench/latency.py --steps 1000 > $O/latency_config2.json || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_w5.json || exit $?
exit $rc
