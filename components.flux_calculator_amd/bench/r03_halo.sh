#!/bin/bash
# Halo tiles vs crossing records + fix-up: the GPU suite, then in-process A/Bs of the same
# build with FCX_OPT_ATMOS_HALO 1 (ref) and 0 (nohalo), fp64 and fp32, bench.py's random map;
# then the default bench line.  Output under gpurun_out/$1 (default r03h).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03h}
mkdir -p $O
AB=components.flux_calculator_amd/bench/inproc_ab.py
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 $AB --opts nohalo:atmos_halo=0 > $O/ab_halo_f64.json || exit $?
timeout -k 10 300 python3 $AB --opts nohalo:atmos_halo=0 --precision f32 > $O/ab_halo_f32.json || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_w5.json || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu --precision f32 > $O/bench_f32.json || exit $?
exit $rc
