// span_probe.hip -- measurement tool (round 6): the Baltic-size step of the three variants
// with every engine's inputs in ONE adjacent host span and its outputs in another, so that an
// engine's phase is one H2D, its kernel, one D2H.  How should the copies be queued for the
// copy engines to run both directions at once?  Schedules (median wall time per step of the
// three engines, each step ended by synchronising every stream):
//   own      each engine's H2D, kernel, D2H on its own stream
//   upq      uploads in call order on one shared upload stream, an event, the kernel and the
//            D2H on the engine's stream
//   upq_dnq  as upq, the downloads on one shared download stream as well
//   single   everything on one stream (no overlap: the sum of the bytes)
//   halves   own, every engine's cells in two halves (two H2D / kernel / D2H rounds)
// Sizes: CCLM 10 inputs / 7 outputs, MOM5 11 / 7, RCO 5 / 6 arrays of 32,768 fp64 cells.
//
//   hipcc --offload-arch=gfx950 -O2 span_probe.hip -o span_probe && ./span_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
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

// a stand-in for the flux kernel: every output array = a sum of the inputs (reads all, writes all)
__global__ void touch(const double *in, int nin, double *out, int nout, int n, int64_t lo, int64_t hi) {
  const int64_t j = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= hi) return;
  double s = 0.0;
  for (int k = 0; k < nin; ++k) s += in[(int64_t)k * n + j];
  for (int k = 0; k < nout; ++k) out[(int64_t)k * n + j] = s + k;
}

struct Eng {
  int nin, nout;
  double *h_in, *h_out, *d_in, *d_out;
  hipStream_t s;
  hipEvent_t ev;
};

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 32768;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 300;
  const int shape[3][2] = {{10, 7}, {11, 7}, {5, 6}};
  std::vector<Eng> es(3);
  hipStream_t s_up, s_dn;
  CHECK(hipStreamCreateWithFlags(&s_up, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s_dn, hipStreamNonBlocking));
  for (int i = 0; i < 3; ++i) {
    Eng &e = es[i];
    e.nin = shape[i][0];
    e.nout = shape[i][1];
    CHECK(hipHostMalloc((void **)&e.h_in, (size_t)e.nin * n * 8, hipHostMallocDefault));
    CHECK(hipHostMalloc((void **)&e.h_out, (size_t)e.nout * n * 8, hipHostMallocDefault));
    CHECK(hipMalloc((void **)&e.d_in, (size_t)e.nin * n * 8));
    CHECK(hipMalloc((void **)&e.d_out, (size_t)e.nout * n * 8));
    for (size_t k = 0; k < (size_t)e.nin * n; ++k) e.h_in[k] = 1.0;
    CHECK(hipStreamCreateWithFlags(&e.s, hipStreamNonBlocking));
    CHECK(hipEventCreateWithFlags(&e.ev, hipEventDisableTiming));
  }
  auto phase = [&](Eng &e, hipStream_t up, hipStream_t dn, int64_t lo, int64_t hi, bool edge,
                   hipStream_t ks = nullptr) -> hipError_t {
    if (!ks) ks = e.s;  // the kernel's stream
    // [lo, hi) of every array: a strided span (one 2-D copy) unless it is the whole array
    const size_t w = (size_t)(hi - lo) * 8, pitch = (size_t)n * 8;
    hipError_t r = (hi - lo == n) ? hipMemcpyAsync(e.d_in, e.h_in, (size_t)e.nin * pitch, hipMemcpyDefault, up)
                                  : hipMemcpy2DAsync(e.d_in + lo, pitch, e.h_in + lo, pitch, w, e.nin, hipMemcpyDefault, up);
    if (r) return r;
    if (edge) {
      if ((r = hipEventRecord(e.ev, up))) return r;
      if ((r = hipStreamWaitEvent(ks, e.ev, 0))) return r;
    }
    touch<<<(unsigned)((hi - lo + 255) / 256), 256, 0, ks>>>(e.d_in, e.nin, e.d_out, e.nout, n, lo, hi);
    if ((r = hipGetLastError())) return r;
    if (dn != ks) {
      if ((r = hipEventRecord(e.ev, ks))) return r;
      if ((r = hipStreamWaitEvent(dn, e.ev, 0))) return r;
    }
    return (hi - lo == n) ? hipMemcpyAsync(e.h_out, e.d_out, (size_t)e.nout * pitch, hipMemcpyDefault, dn)
                          : hipMemcpy2DAsync(e.h_out + lo, pitch, e.d_out + lo, pitch, w, e.nout, hipMemcpyDefault, dn);
  };
  const char *names[] = {"own", "upq", "upq_dnq", "single", "halves"};
  std::printf("{\"tool\": \"span_probe.hip\", \"cells\": %d, \"reps\": %d, \"schedules\": {", n, reps);
  for (int sc = 0; sc < 5; ++sc) {
    std::vector<double> t;
    for (int r = 0; r < reps + 20; ++r) {
      const double t0 = now_us();
      for (Eng &e : es) {
        hipError_t err = hipSuccess;
        switch (sc) {
          case 0: err = phase(e, e.s, e.s, 0, n, false); break;
          case 1: err = phase(e, s_up, e.s, 0, n, true); break;
          case 2: err = phase(e, s_up, s_dn, 0, n, true); break;
          case 3: err = phase(e, es[0].s, es[0].s, 0, n, false, es[0].s); break;
          case 4:
            err = phase(e, e.s, e.s, 0, n / 2, false);
            if (!err) err = phase(e, e.s, e.s, n / 2, n, false);
            break;
        }
        CHECK(err);
      }
      for (Eng &e : es) CHECK(hipStreamSynchronize(e.s));
      CHECK(hipStreamSynchronize(s_up));
      CHECK(hipStreamSynchronize(s_dn));
      if (r >= 20) t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    std::printf("%s\"%s\": {\"median_us\": %.1f, \"p10_us\": %.1f, \"p90_us\": %.1f}", sc ? ", " : "", names[sc],
                t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
  }
  // check: the outputs of the last step hold the sums
  bool ok = true;
  for (Eng &e : es)
    for (int k = 0; k < e.nout; ++k) ok = ok && e.h_out[(size_t)k * n + 7] == e.nin + k;
  std::printf("}, \"outputs_ok\": %s}\n", ok ? "true" : "false");
  return ok ? 0 : 2;
}
