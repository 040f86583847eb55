set -e
mkdir -p gpurun_out/remap_ab
for r in 1 2; do
for v in ref chunk256 chunk1024 chunk2048; do
  if [ $v = ref ]; then L=components.flux_calculator_amd/lib/libfcx.so; else L=ab/$v/libfcx.so; fi
  FCX_LIBRARY=$L timeout -k 10 200 python components.flux_calculator_amd/bench/remap_bench.py --rounds 5 > gpurun_out/remap_ab/${v}_r$r.json
done
done
