#!/bin/bash
# Round-2 evidence with the final build, from the repo root (one MI355X): the default bench
# with the driver's arguments (timed), the rocprof kernel statistics of the same command, the
# request-size PMC passes of the default workload (exact read bytes; WRITE_SIZE), and the
# T = 2, fp32 and bias lines.  Output under gpurun_out/ev2/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/ev2
mkdir -p $O
s=$(date +%s.%N)
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_w5.json
e=$(date +%s.%N)
echo "{\"wall_s\": $(python3 -c "print(round($e - $s, 1))")}" > $O/bench_w5_wall.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_under_rocprof.json
bash components.flux_calculator_amd/bench/pmc_bytes.sh $O/pmc_t1 -- python3 bench.py --steps 5 --warmup 1 --no-cpu --config4 0 --other-map 0
bash components.flux_calculator_amd/bench/pmc_bytes.sh $O/pmc_t2 -- python3 bench.py --steps 3 --warmup 1 --no-cpu --config4 0 --other-map 0 --types 2
timeout -k 10 300 python3 bench.py --no-cpu --types 2 > $O/bench_T2.json
timeout -k 10 300 python3 bench.py --no-cpu --precision f32 > $O/bench_f32.json
timeout -k 10 300 python3 bench.py --no-cpu --bias > $O/bench_bias.json
echo done > $O/DONE
