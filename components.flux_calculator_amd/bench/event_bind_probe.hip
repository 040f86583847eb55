// event_bind_probe.hip -- what does a timing-event pair around one kernel of a back-to-back
// sequence cost, recorded as markers (hipEventRecord before and after the launch) against
// bound to the launch itself (hipExtLaunchKernelGGL start/stop events)?  Three streaming
// kernels per "step" (1.6 GB each, the shape of the bench's step); not part of the product.
//   hipcc --offload-arch=gfx950 -O3 event_bind_probe.hip -o event_bind_probe && ./event_bind_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
      return 1;                                                          \
    }                                                                    \
  } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void stream_kernel(const d2 *__restrict__ a, d2 *__restrict__ b, long n2) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n2) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i) * 1.0000001, b + i);
}

int main() {
  const long n2 = 50L << 20;  // 50M d2 = 800 MB in, 800 MB out per kernel
  d2 *in[3], *out[3];
  for (int k = 0; k < 3; ++k) {
    CHECK(hipMalloc(&in[k], n2 * sizeof(d2)));
    CHECK(hipMalloc(&out[k], n2 * sizeof(d2)));
    CHECK(hipMemset(in[k], 0, n2 * sizeof(d2)));
  }
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  const int steps = 200;
  hipEvent_t ev[2 * steps];
  for (auto &e : ev) CHECK(hipEventCreate(&e));
  const dim3 grid((unsigned)((n2 + 255) / 256)), block(256);
  const char *names[3] = {"no events", "marker pair around kernel 2", "pair bound to kernel 2"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 3; ++mode) {
      auto step = [&](int t, bool timed) {
        hipLaunchKernelGGL(stream_kernel, grid, block, 0, s, in[0], out[0], n2);
        if (timed && mode == 1) (void)hipEventRecord(ev[2 * t], s);
        if (timed && mode == 2)
          hipExtLaunchKernelGGL(stream_kernel, grid, block, 0, s, ev[2 * t], ev[2 * t + 1], 0, in[1], out[1], n2);
        else
          hipLaunchKernelGGL(stream_kernel, grid, block, 0, s, in[1], out[1], n2);
        if (timed && mode == 1) (void)hipEventRecord(ev[2 * t + 1], s);
        hipLaunchKernelGGL(stream_kernel, grid, block, 0, s, in[2], out[2], n2);
      };
      for (int t = 0; t < 100; ++t) step(0, false);
      CHECK(hipStreamSynchronize(s));
      const auto t0 = std::chrono::steady_clock::now();
      for (int t = 0; t < steps; ++t) step(t, true);
      CHECK(hipStreamSynchronize(s));
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      double kms = 0;
      if (mode) {
        for (int t = 0; t < steps; ++t) {
          float x;
          CHECK(hipEventElapsedTime(&x, ev[2 * t], ev[2 * t + 1]));
          kms += x;
        }
        kms /= steps;
      }
      printf("{\"rep\": %d, \"mode\": \"%s\", \"us_per_step\": %.2f, \"kernel2_us\": %.2f}\n", rep, names[mode],
             ms * 1e3 / steps, kms * 1e3);
    }
  return 0;
}
