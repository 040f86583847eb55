// mix_probe.hip -- can a kernel's own reads of mapped host memory (the zero-copy inputs) and a
// copy-engine download (hipMemcpyAsync device -> page-locked host) use the two directions of
// the host link at once?  (measurement tool).  At the Baltic step's
// sizes (6.8 MB of inputs up, 5.2 MB of outputs down, the three variants), median wall time:
//   read     a kernel streams the inputs from mapped host memory (sums into device memory)
//   dma_d2h  hipMemcpyAsync(hipMemcpyDefault) of the outputs, device -> host
//   both     the two at once on two non-blocking streams
//   zc       one kernel reads the inputs and writes the outputs to mapped host memory (the
//            zero-copy step's traffic)
//
//   hipcc --offload-arch=gfx950 -O2 mix_probe.hip -o mix_probe && ./mix_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// every lane sums its float4s of `in` (grid-stride) and writes one value to `sink` (device);
// with `out` set it also writes out[i] = in[i] for i < n_out (mapped host memory)
__global__ __launch_bounds__(256) void read_kernel(const float4 *__restrict__ in, int64_t n_in, float *__restrict__ sink,
                                                    float4 *__restrict__ out, int64_t n_out) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (int64_t i = i0; i < n_in; i += stride) {
    const float4 v = in[i];
    acc += v.x + v.y + v.z + v.w;
    if (out && i < n_out) out[i] = v;
  }
  sink[i0] = acc;
}

int main() {
  const size_t up = 6815744, down = 5242880;  // bytes: the Baltic step of the three variants
  const int reps = 200;
  float4 *hin = nullptr, *hout = nullptr, *dout = nullptr;
  float *sink = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void **>(&hin), up, hipHostMallocDefault));
  CHECK(hipHostMalloc(reinterpret_cast<void **>(&hout), down, hipHostMallocDefault));
  CHECK(hipMalloc(reinterpret_cast<void **>(&dout), down));
  std::memset(hin, 0, up);
  CHECK(hipMemset(dout, 0, down));
  float4 *hin_d = nullptr, *hout_d = nullptr;  // device-side addresses of the mapped blocks
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&hin_d), hin, 0));
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&hout_d), hout, 0));
  const int blocks = 1024, threads = 256;
  CHECK(hipMalloc(reinterpret_cast<void **>(&sink), sizeof(float) * blocks * threads));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int64_t n_in = (int64_t)(up / sizeof(float4)), n_out = (int64_t)(down / sizeof(float4));

  auto time_it = [&](int what) -> double {  // 0 read, 1 dma_d2h, 2 both, 3 zc
    std::vector<double> t;
    for (int r = 0; r < reps + 20; ++r) {
      const double t0 = now_us();
      if (what == 0 || what == 2)
        hipLaunchKernelGGL(read_kernel, dim3(blocks), dim3(threads), 0, s1, hin_d, n_in, sink, nullptr, 0);
      if (what == 1 || what == 2) (void)hipMemcpyAsync(hout, dout, down, hipMemcpyDefault, s2);
      if (what == 3)
        hipLaunchKernelGGL(read_kernel, dim3(blocks), dim3(threads), 0, s1, hin_d, n_in, sink, hout_d, n_out);
      (void)hipStreamSynchronize(s1);
      (void)hipStreamSynchronize(s2);
      if (r >= 20) t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  const char *names[4] = {"read", "dma_d2h", "both", "zc"};
  const double bytes[4] = {(double)up, (double)down, (double)(up + down), (double)(up + down)};
  std::printf("{");
  for (int w = 0; w < 4; ++w) {
    const double us = time_it(w);
    CHECK(hipGetLastError());
    std::printf("%s\"%s_us\": %.1f, \"%s_GBps\": %.1f", w ? ", " : "", names[w], us, names[w], bytes[w] / us / 1e3);
  }
  std::printf("}\n");
  CHECK(hipStreamDestroy(s1));
  CHECK(hipStreamDestroy(s2));
  CHECK(hipFree(sink));
  CHECK(hipFree(dout));
  CHECK(hipHostFree(hin));
  CHECK(hipHostFree(hout));
  return 0;
}
