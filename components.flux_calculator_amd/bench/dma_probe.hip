// dma_probe.hip -- the host link as libfcx's staging transfers use it (measurement tool):
// hipMemcpyAsync between page-locked host memory (hipHostMalloc) and device memory on
// non-blocking streams, H2D alone, D2H alone, and both at once on two streams, at the
// Baltic step's sizes (6.8 MB up, 5.2 MB down: the three variants; 2.6 / 1.8 MB: CCLM) and
// at 256 MiB.  Median wall time of `reps` repetitions, each ended by synchronising both
// streams.  (bench/link_probe.py measures the same with torch copies.)
//
//   hipcc --offload-arch=gfx950 -O2 dma_probe.hip -o dma_probe && ./dma_probe [default|noncoherent|portable] [default]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <chrono>
#include <cstdio>
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

int main(int argc, char **argv) {
  // argv[1]: host allocation flags -- "default" (hipHostMallocDefault, as the staging arena),
  // "noncoherent" (hipHostMallocNonCoherent), "portable" (hipHostMallocPortable); argv[2]:
  // "default" = the copies' kind hipMemcpyDefault instead of the explicit direction
  const char *mode = argc > 1 ? argv[1] : "default";
  const bool kind_default = argc > 2 && std::string(argv[2]) == "default";
  unsigned flags = hipHostMallocDefault;
  if (std::string(mode) == "noncoherent") flags = hipHostMallocNonCoherent;
  if (std::string(mode) == "portable") flags = hipHostMallocPortable;
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  struct Case {
    const char *name;
    size_t up, down;
    int reps;
  };
  const Case cases[] = {{"cclm_step", 2621440, 1835008, 400},
                        {"three_variants_step", 6815744, 5242880, 300},
                        {"256MiB", size_t(256) << 20, size_t(256) << 20, 10}};
  std::printf("{\"tool\": \"dma_probe.hip\", \"host_alloc\": \"%s\", \"kind\": \"%s\", \"cases\": [", mode,
              kind_default ? "hipMemcpyDefault" : "explicit");
  bool first = true;
  for (const Case &c : cases) {
    void *hu, *hd, *du, *dd;
    CHECK(hipHostMalloc(&hu, c.up, flags));
    CHECK(hipHostMalloc(&hd, c.down, flags));
    CHECK(hipMalloc(&du, c.up));
    CHECK(hipMalloc(&dd, c.down));
    CHECK(hipMemset(du, 0, c.up));
    CHECK(hipMemset(dd, 0, c.down));
    double res[3];
    for (int dir = 0; dir < 3; ++dir) {  // 0 up, 1 down, 2 both
      std::vector<double> t;
      for (int r = 0; r < c.reps + 5; ++r) {
        const double t0 = now_us();
        if (dir != 1) CHECK(hipMemcpyAsync(du, hu, c.up, kind_default ? hipMemcpyDefault : hipMemcpyHostToDevice, s1));
        if (dir != 0) CHECK(hipMemcpyAsync(hd, dd, c.down, kind_default ? hipMemcpyDefault : hipMemcpyDeviceToHost, s2));
        CHECK(hipStreamSynchronize(s1));
        CHECK(hipStreamSynchronize(s2));
        if (r >= 5) t.push_back(now_us() - t0);
      }
      std::sort(t.begin(), t.end());
      res[dir] = t[t.size() / 2];
    }
    std::printf("%s{\"case\": \"%s\", \"h2d_bytes\": %zu, \"d2h_bytes\": %zu, \"h2d_us\": %.1f, \"d2h_us\": %.1f, "
                "\"both_us\": %.1f, \"h2d_GBps\": %.1f, \"d2h_GBps\": %.1f, \"both_GBps\": %.1f}",
                first ? "" : ", ", c.name, c.up, c.down, res[0], res[1], res[2], c.up / res[0] / 1e3,
                c.down / res[1] / 1e3, (c.up + c.down) / res[2] / 1e3);
    first = false;
    CHECK(hipHostFree(hu));
    CHECK(hipHostFree(hd));
    CHECK(hipFree(du));
    CHECK(hipFree(dd));
  }
  std::printf("]}\n");
  return 0;
}
