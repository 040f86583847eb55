#!/bin/bash
# round 6: kernel + memory-copy trace of span_probe's schedules on portable host memory (the
# device buffers written first), to see where the duplex schedule's time goes
set -euo pipefail
O=${1:-gpurun_out/r06/spantrace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 components.flux_calculator_amd/lib/probe/span_probe 32768 300 portable > $O/span_probe_portable.json
cat $O/span_probe_portable.json
for sc in duplex single both_alone; do
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace_$sc -o run -- \
    components.flux_calculator_amd/lib/probe/span_probe 32768 30 portable $sc > $O/probe_$sc.json
done
find $O -name "*.csv" | head -20
