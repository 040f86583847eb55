# A/B of the in-launch crossing completion (profiles/r02/xcomplete_ab/xcomplete.patch applied;
# not kept: the option it sets no longer exists in the product build).
set -o pipefail
mkdir -p gpurun_out/xc
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_fp32.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "long_segments or fused_accumulation" > gpurun_out/xc/tests.log 2>&1 || exit 1
for r in 1 2; do for x in 0 1; do
timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 5 --config4 0 --other-map 0 --cross-complete $x > gpurun_out/xc/bench_x${x}_r$r.json 2>> gpurun_out/xc/bench.err || exit 2
done; done
for x in 0 1; do
timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 5 --config4 0 --other-map 0 --precision f32 --cross-complete $x > gpurun_out/xc/bench_f32_x${x}.json 2>> gpurun_out/xc/bench.err || exit 3
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/xc/gpu_suite.log 2>&1 || exit 4
