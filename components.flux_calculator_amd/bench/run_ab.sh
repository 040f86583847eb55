#!/bin/bash
# A/B: libs x max_blocks, interleaved rounds; one JSON line per run into gpurun_out/ab/
set -e
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in $LIBS; do
    for mb in $MBS; do
      FCX_LIBRARY=ab/$lib/libfcx.so timeout -k 10 120 python bench.py --no-cpu --max-blocks $mb $EXTRA > gpurun_out/ab/${lib}_mb${mb}_r$r.json
    done
  done
done
