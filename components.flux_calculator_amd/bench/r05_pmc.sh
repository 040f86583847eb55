#!/bin/bash
# round 5 counters with the round's kernels: HBM request bytes (pmc_bytes.sh: read-request
# sizes, then WRITE_SIZE) of the fp64 T = 1 and fp32 group launches, and the SQ issue /
# LDS-conflict counters of the same (two passes of 8 SQ counters), each pass its own run
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/pmc; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu --e2e 0 --other-map 0 --config4 0"
B=components.flux_calculator_amd/bench
bash $B/pmc_bytes.sh $O/pmc_t1 -- python3 bench.py $A
bash $B/pmc_bytes.sh $O/pmc_f32 -- python3 bench.py $A --precision f32
for spec in "t1|$A" "f32|$A --precision f32"; do
  N=${spec%%|*}; ARGS=${spec#*|}
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    --kernel-trace --output-format csv -d $O/sq_$N/sq -o run -- python3 bench.py $ARGS > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $O/sq_$N/sq2 -o run -- python3 bench.py $ARGS > /dev/null
done
echo done > $O/DONE
