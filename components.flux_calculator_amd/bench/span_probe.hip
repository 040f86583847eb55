// span_probe.hip -- measurement tool (round 6): the Baltic-size step of the three variants
// with every engine's inputs in ONE adjacent host span and its outputs in another, so that an
// engine's phase is one H2D, its kernel, one D2H.  How should the copies be queued for the
// copy engines to run both directions at once?  Median wall time per step of the three
// engines (each step ended by synchronising every stream used), for these schedules:
//   up_alone / down_alone / both_alone   the 3 engines' inputs up (one copy each), outputs
//                                        down, both directions at once on two streams (the
//                                        link's own floors at these sizes, no kernels)
//   own        each engine's H2D, kernel, D2H on its own stream
//   single     everything on one stream, engine after engine
//   phased     one stream: the three uploads, the three kernels, the three downloads
//   duplex     uploads in order on stream A (an event after each); on stream B each engine
//              waits for its upload, runs its kernel and its download -- engine k's download
//              overlaps the later engines' uploads
//   duplex_k   as duplex, the kernels on stream A after each upload (no cross-stream wait
//              before a kernel; B waits for the kernel's event before the download)
//   one_span   all three engines' inputs as ONE copy, the kernels, ONE download
// argv: cells (32768), reps (300), host flags: default | mapped | portable | mapped_portable
// (hipHostMalloc flags; round 6: device->host copies into default or mapped memory run at
// ~23 GB/s, into portable memory at ~52 GB/s -- bench/d2h_flags_probe.hip).
//
//   hipcc --offload-arch=gfx950 -O2 span_probe.hip -o span_probe && ./span_probe 32768 300 mapped
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
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

// a stand-in for the flux kernel: every output array = a sum of the inputs (reads all, writes all)
__global__ void touch(const double *in, int nin, double *out, int nout, int n) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int k = 0; k < nin; ++k) s += in[(int64_t)k * n + j];
  for (int k = 0; k < nout; ++k) out[(int64_t)k * n + j] = s + k;
}

struct Eng {
  int nin, nout;
  char *h_in, *h_out, *d_in, *d_out;
  size_t b_in, b_out;
  hipStream_t s;
  hipEvent_t ev_up, ev_k;
};

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 32768;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 300;
  const std::string hf = argc > 3 ? argv[3] : "default";
  const unsigned hflags = hf == "mapped" ? hipHostMallocMapped
                          : hf == "portable" ? hipHostMallocPortable
                          : hf == "mapped_portable" ? (hipHostMallocMapped | hipHostMallocPortable)
                                                    : hipHostMallocDefault;
  const int shape[3][2] = {{10, 7}, {11, 7}, {5, 6}};
  std::vector<Eng> es(3);
  hipStream_t sa, sb;
  CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  // one host slab for every engine: inputs of all engines, then outputs (the reference's
  // allocation order), so that one_span can move them as single copies
  size_t tin = 0, tout = 0;
  for (int i = 0; i < 3; ++i) {
    es[i].nin = shape[i][0];
    es[i].nout = shape[i][1];
    es[i].b_in = (size_t)es[i].nin * n * 8;
    es[i].b_out = (size_t)es[i].nout * n * 8;
    tin += es[i].b_in;
    tout += es[i].b_out;
  }
  char *h, *d;
  CHECK(hipHostMalloc((void **)&h, tin + tout, hflags));
  CHECK(hipMalloc((void **)&d, tin + tout));
  CHECK(hipMemset(d, 0, tin + tout));  // (D2H out of never-written device pages runs ~5x slower)
  size_t oi = 0, oo = tin;
  for (Eng &e : es) {
    e.h_in = h + oi, e.d_in = d + oi, oi += e.b_in;
    e.h_out = h + oo, e.d_out = d + oo, oo += e.b_out;
    for (size_t k = 0; k < e.b_in / 8; ++k) reinterpret_cast<double *>(e.h_in)[k] = 1.0;
    CHECK(hipStreamCreateWithFlags(&e.s, hipStreamNonBlocking));
    CHECK(hipEventCreateWithFlags(&e.ev_up, hipEventDisableTiming));
    CHECK(hipEventCreateWithFlags(&e.ev_k, hipEventDisableTiming));
  }
  auto up = [&](Eng &e, hipStream_t s) { CHECK(hipMemcpyAsync(e.d_in, e.h_in, e.b_in, hipMemcpyDefault, s)); };
  auto down = [&](Eng &e, hipStream_t s) { CHECK(hipMemcpyAsync(e.h_out, e.d_out, e.b_out, hipMemcpyDefault, s)); };
  auto kern = [&](Eng &e, hipStream_t s) {
    touch<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(reinterpret_cast<const double *>(e.d_in), e.nin,
                                                         reinterpret_cast<double *>(e.d_out), e.nout, n);
    CHECK(hipGetLastError());
  };
  const char *names[] = {"up_alone", "down_alone", "both_alone", "own", "single", "phased", "duplex", "duplex_k",
                         "one_span"};
  const int ns = sizeof(names) / sizeof(names[0]);
  std::printf("{\"tool\": \"span_probe.hip\", \"cells\": %d, \"reps\": %d, \"host\": \"%s\", \"in_bytes\": %zu, "
              "\"out_bytes\": %zu, \"schedules\": {",
              n, reps, hf.c_str(), tin, tout);
  const std::string only = argc > 4 ? argv[4] : "";  // a comma list of schedules (default: all)
  bool first = true;
  for (int sc = 0; sc < ns; ++sc) {
    if (!only.empty() && ("," + only + ",").find("," + std::string(names[sc]) + ",") == std::string::npos) continue;
    std::vector<double> t;
    for (int r = 0; r < reps + 20; ++r) {
      const double t0 = now_us();
      switch (sc) {
        case 0:
          for (Eng &e : es) up(e, sa);
          break;
        case 1:
          for (Eng &e : es) down(e, sb);
          break;
        case 2:
          for (Eng &e : es) up(e, sa);
          for (Eng &e : es) down(e, sb);
          break;
        case 3:
          for (Eng &e : es) up(e, e.s), kern(e, e.s), down(e, e.s);
          break;
        case 4:
          for (Eng &e : es) up(e, sa), kern(e, sa), down(e, sa);
          break;
        case 5:
          for (Eng &e : es) up(e, sa);
          for (Eng &e : es) kern(e, sa);
          for (Eng &e : es) down(e, sa);
          break;
        case 6:
          for (Eng &e : es) {
            up(e, sa);
            CHECK(hipEventRecord(e.ev_up, sa));
          }
          for (Eng &e : es) {
            CHECK(hipStreamWaitEvent(sb, e.ev_up, 0));
            kern(e, sb);
            down(e, sb);
          }
          break;
        case 7:
          for (Eng &e : es) {
            up(e, sa);
            kern(e, sa);
            CHECK(hipEventRecord(e.ev_k, sa));
          }
          for (Eng &e : es) {
            CHECK(hipStreamWaitEvent(sb, e.ev_k, 0));
            down(e, sb);
          }
          break;
        case 8:
          CHECK(hipMemcpyAsync(d, h, tin, hipMemcpyDefault, sa));
          for (Eng &e : es) kern(e, sa);
          CHECK(hipMemcpyAsync(h + tin, d + tin, tout, hipMemcpyDefault, sa));
          break;
      }
      for (Eng &e : es) CHECK(hipStreamSynchronize(e.s));
      CHECK(hipStreamSynchronize(sa));
      CHECK(hipStreamSynchronize(sb));
      if (r >= 20) t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    std::printf("%s\"%s\": {\"median_us\": %.1f, \"p10_us\": %.1f, \"p90_us\": %.1f}", first ? "" : ", ", names[sc],
                t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
    first = false;
  }
  bool ok = true;
  for (Eng &e : es)
    for (int k = 0; k < e.nout; ++k) ok = ok && reinterpret_cast<double *>(e.h_out)[(size_t)k * n + 7] == e.nin + k;
  std::printf("}, \"outputs_ok\": %s}\n", ok ? "true" : "false");
  return ok ? 0 : 2;
}
