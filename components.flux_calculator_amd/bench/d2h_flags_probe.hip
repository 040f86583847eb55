// d2h_flags_probe.hip -- measurement tool (round 6): why a device->host copy into page-locked
// memory runs at ~10 GB/s in one case and ~50 GB/s in another (span_probe, profiles/r06/).
// For each hipHostMalloc flag set: the Baltic step's 6.8 MB of inputs up and 5.2 MB of
// outputs down at offsets inside ONE host allocation (the fcx_host_malloc slab layout), as
// one copy per direction or three (one per engine), alone and both directions at once on two
// streams; the device buffer written by a kernel beforehand or not.  Median wall time of
// `reps` repetitions, each ended by synchronising both streams.
//
//   hipcc --offload-arch=gfx950 -O2 d2h_flags_probe.hip -o d2h_flags_probe && ./d2h_flags_probe
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

__global__ void fill(double *p, size_t n, double v) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v + (double)i;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const size_t tin = 6815744, tout = 5242880;
  const size_t parts_in[3] = {2621440, 2883584, 1310720}, parts_out[3] = {1835008, 1835008, 1572864};
  struct Flag {
    const char *name;
    unsigned f;
  };
  const Flag flags[] = {{"default", hipHostMallocDefault},
                        {"mapped", hipHostMallocMapped},
                        {"portable", hipHostMallocPortable},
                        {"coherent", hipHostMallocCoherent},
                        {"noncoherent", hipHostMallocNonCoherent},
                        {"mapped_noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent},
                        {"mapped_portable", hipHostMallocMapped | hipHostMallocPortable}};
  hipStream_t sa, sb;
  CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  char *d;
  CHECK(hipMalloc((void **)&d, tin + tout));
  std::printf("{\"tool\": \"d2h_flags_probe.hip\", \"reps\": %d, \"in_bytes\": %zu, \"out_bytes\": %zu, \"flags\": {", reps,
              tin, tout);
  bool first = true;
  for (const Flag &fl : flags) {
    char *h = nullptr;
    if (hipHostMalloc((void **)&h, tin + tout, fl.f) != hipSuccess) {
      (void)hipGetLastError();
      continue;
    }
    memset(h, 0, tin + tout);
    fill<<<(unsigned)((tin + tout) / 8 / 256 + 1), 256>>>(reinterpret_cast<double *>(d), (tin + tout) / 8, 1.0);
    CHECK(hipDeviceSynchronize());
    const char *cases[] = {"up1", "up3", "down1", "down3", "both1", "both3", "down1_explicit"};
    std::printf("%s\"%s\": {", first ? "" : ", ", fl.name);
    first = false;
    for (int c = 0; c < 7; ++c) {
      std::vector<double> t;
      for (int r = 0; r < reps + 10; ++r) {
        const double t0 = now_us();
        const bool up = c == 0 || c == 1 || c == 4 || c == 5, down = !(c == 0 || c == 1), three = c == 1 || c == 3 || c == 5;
        if (up) {
          if (three) {
            size_t o = 0;
            for (size_t p : parts_in) {
              CHECK(hipMemcpyAsync(d + o, h + o, p, hipMemcpyDefault, sa));
              o += p;
            }
          } else {
            CHECK(hipMemcpyAsync(d, h, tin, hipMemcpyDefault, sa));
          }
        }
        if (down) {
          const hipMemcpyKind k = c == 6 ? hipMemcpyDeviceToHost : hipMemcpyDefault;
          if (three) {
            size_t o = tin;
            for (size_t p : parts_out) {
              CHECK(hipMemcpyAsync(h + o, d + o, p, k, sb));
              o += p;
            }
          } else {
            CHECK(hipMemcpyAsync(h + tin, d + tin, tout, k, sb));
          }
        }
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
