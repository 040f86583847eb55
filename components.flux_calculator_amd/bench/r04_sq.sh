#!/bin/bash
# SQ issue/stall counters of the group kernel (fp64 T = 1, fp32, T = 2): one pass of 8 SQ
# counters and one of GRBM_GUI_ACTIVE (clock) per workload, separate runs
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/sq; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu --e2e 0 --other-map 0 --config4 0"
for spec in "t1|$A" "f32|$A --precision f32" "t2|$A --types 2"; do
  N=${spec%%|*}; ARGS=${spec#*|}
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    --kernel-trace --output-format csv -d $O/$N/sq -o run -- python3 bench.py $ARGS > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $O/$N/sq2 -o run -- python3 bench.py $ARGS > /dev/null
done
