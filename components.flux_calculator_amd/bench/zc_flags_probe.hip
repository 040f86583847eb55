// zc_flags_probe.hip -- measurement tool (round 6): the host link as the KERNELS use it
// (zero-copy: loads and stores to page-locked host memory through its device address) and as
// the copy engines use it, by hipHostMalloc flag set.  The Baltic step's traffic: 6.8 MB of
// inputs read, 5.2 MB of outputs written.  Per flag set, median wall time of `reps`
// repetitions, each synchronised:
//   k_read       a kernel reads the inputs from host memory (sums them into device memory)
//   k_write      a kernel writes the outputs to host memory
//   k_readwrite  one kernel reads the inputs and writes the outputs (the zero-copy step)
//   dma_up / dma_down / dma_both   the same bytes by hipMemcpyAsync (one copy each way;
//                                  both: two streams at once)
// Host memory is written by the CPU first (never-touched pages are slow to DMA into).
//
//   hipcc --offload-arch=gfx950 -O2 zc_flags_probe.hip -o zc_flags_probe && ./zc_flags_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// cells of `nin` input arrays (host) summed, `nout` output arrays (host) written; one cell per
// lane, 16-B accesses (two cells)
__global__ void zc_step(const double2 *in, int nin, double2 *out, int nout, double2 *dev_sink, int n2) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n2) return;
  double2 s = make_double2(0.0, 0.0);
  for (int k = 0; k < nin; ++k) {
    const double2 v = in[(size_t)k * n2 + j];
    s.x += v.x;
    s.y += v.y;
  }
  if (nout == 0) {
    dev_sink[j] = s;
    return;
  }
  for (int k = 0; k < nout; ++k) out[(size_t)k * n2 + j] = make_double2(s.x + k, s.y + k);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const int n = 32768, nin = 26, nout = 20;  // 26 x 256 KiB = 6.8 MB in, 20 x 256 KiB = 5.2 MB out
  const size_t tin = (size_t)nin * n * 8, tout = (size_t)nout * n * 8;
  struct Flag {
    const char *name;
    unsigned f;
  };
  const Flag flags[] = {{"mapped", hipHostMallocMapped},
                        {"mapped_portable", hipHostMallocMapped | hipHostMallocPortable},
                        {"mapped_noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent},
                        {"mapped_coherent", hipHostMallocMapped | hipHostMallocCoherent}};
  hipStream_t sa, sb;
  CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  char *d;
  CHECK(hipMalloc((void **)&d, tin + tout));
  CHECK(hipMemset(d, 0, tin + tout));
  double2 *sink;
  CHECK(hipMalloc((void **)&sink, (size_t)n * 8));
  std::printf("{\"tool\": \"zc_flags_probe.hip\", \"reps\": %d, \"in_bytes\": %zu, \"out_bytes\": %zu, \"flags\": {", reps,
              tin, tout);
  bool first = true;
  for (const Flag &fl : flags) {
    char *h = nullptr, *hd = nullptr;
    if (hipHostMalloc((void **)&h, tin + tout, fl.f) != hipSuccess) {
      (void)hipGetLastError();
      continue;
    }
    CHECK(hipHostGetDevicePointer((void **)&hd, h, 0));
    for (size_t i = 0; i < (tin + tout) / 8; ++i) reinterpret_cast<double *>(h)[i] = 1.0;
    const char *cases[] = {"k_read", "k_write", "k_readwrite", "dma_up", "dma_down", "dma_both"};
    std::printf("%s\"%s\": {", first ? "" : ", ", fl.name);
    first = false;
    const int n2 = n / 2, blocks = (n2 + 255) / 256;
    for (int c = 0; c < 6; ++c) {
      std::vector<double> t;
      for (int r = 0; r < reps + 10; ++r) {
        const double t0 = now_us();
        switch (c) {
          case 0:
            zc_step<<<blocks, 256, 0, sa>>>(reinterpret_cast<const double2 *>(hd), nin, nullptr, 0, sink, n2);
            break;
          case 1:
            zc_step<<<blocks, 256, 0, sa>>>(reinterpret_cast<const double2 *>(d), 1,
                                             reinterpret_cast<double2 *>(hd + tin), nout, sink, n2);
            break;
          case 2:
            zc_step<<<blocks, 256, 0, sa>>>(reinterpret_cast<const double2 *>(hd), nin,
                                             reinterpret_cast<double2 *>(hd + tin), nout, sink, n2);
            break;
          case 3:
            CHECK(hipMemcpyAsync(d, h, tin, hipMemcpyDefault, sa));
            break;
          case 4:
            CHECK(hipMemcpyAsync(h + tin, d + tin, tout, hipMemcpyDefault, sb));
            break;
          case 5:
            CHECK(hipMemcpyAsync(d, h, tin, hipMemcpyDefault, sa));
            CHECK(hipMemcpyAsync(h + tin, d + tin, tout, hipMemcpyDefault, sb));
            break;
        }
        CHECK(hipGetLastError());
        CHECK(hipStreamSynchronize(sa));
        CHECK(hipStreamSynchronize(sb));
        if (r >= 10) t.push_back(now_us() - t0);
      }
      std::sort(t.begin(), t.end());
      std::printf("%s\"%s\": %.1f", c ? ", " : "", cases[c], t[t.size() / 2]);
    }
    std::printf("}");
    CHECK(hipHostFree(h));
  }
  std::printf("}}\n");
  return 0;
}
