set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/arm1; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t1 -o run -- python3 $B/arm_ab.py --arms "halo:random;nohalo:random:atmos_halo=0;periodic:periodic" --rounds 6 > $O/t1.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t2 -o run -- python3 $B/arm_ab.py --types 2 --arms "random:random;periodic:periodic" --rounds 6 > $O/t2.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/f32 -o run -- python3 $B/arm_ab.py --precision f32 --arms "halo:random;nohalo:random:atmos_halo=0;periodic:periodic" --rounds 6 > $O/f32.json
for x in t1 t2 f32; do python3 $B/split_trace.py $O/$x/run_kernel_trace.csv $O/$x.json > $O/${x}_split.json; done
