// stream_probe.hip -- what HBM bandwidth does an R-in / W-out fp64 SoA stream reach on
// MI355X?  Trivial arithmetic, same access pattern as the fused flux kernel (CCLM: 10 input
// arrays, 7 output arrays).  Used to set the achievable ceiling the flux kernel is judged
// against; not part of the product.
//   hipcc --offload-arch=gfx950 -O3 stream_probe.hip -o stream_probe && ./stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) {                                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                                        \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

struct Ptrs {
  const double *in[32];
  double *out[32];
};

template <int R, int W, int C, bool NT>
__global__ __launch_bounds__(256) void probe(Ptrs p, long n) {
  const long units = n / C;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long u = (long)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += stride) {
    double acc[C];
#pragma unroll
    for (int i = 0; i < C; ++i) acc[i] = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (C == 2) {
        d2 t = NT ? __builtin_nontemporal_load(reinterpret_cast<const d2 *>(p.in[r]) + u)
                       : reinterpret_cast<const d2 *>(p.in[r])[u];
        acc[0] += t[0];
        acc[1] += t[1];
      } else if constexpr (C == 4) {
        const d2 *q = reinterpret_cast<const d2 *>(p.in[r]) + 2 * u;
        d2 a = NT ? __builtin_nontemporal_load(q) : q[0];
        d2 b = NT ? __builtin_nontemporal_load(q + 1) : q[1];
        acc[0] += a[0]; acc[1] += a[1]; acc[2] += b[0]; acc[3] += b[1];
      } else {
        acc[0] += NT ? __builtin_nontemporal_load(p.in[r] + u) : p.in[r][u];
      }
    }
    if constexpr (W == 0) {  // read-only: keep the loads alive without a real store stream
      bool hit = false;
#pragma unroll
      for (int i = 0; i < C; ++i) hit = hit || acc[i] == 1234.5;
      if (hit) p.out[0][u] = acc[0];
    }
#pragma unroll
    for (int w = 0; w < W; ++w) {
      if constexpr (C == 2) {
        d2 t = d2{acc[0] * (w + 1), acc[1] * (w + 1)};
        if (NT) __builtin_nontemporal_store(t, reinterpret_cast<d2 *>(p.out[w]) + u);
        else reinterpret_cast<d2 *>(p.out[w])[u] = t;
      } else if constexpr (C == 4) {
        d2 *q = reinterpret_cast<d2 *>(p.out[w]) + 2 * u;
        d2 a = d2{acc[0] * (w + 1), acc[1] * (w + 1)};
        d2 b = d2{acc[2] * (w + 1), acc[3] * (w + 1)};
        if (NT) { __builtin_nontemporal_store(a, q); __builtin_nontemporal_store(b, q + 1); }
        else { q[0] = a; q[1] = b; }
      } else {
        if (NT) __builtin_nontemporal_store(acc[0] * (w + 1), p.out[w] + u);
        else p.out[w][u] = acc[0] * (w + 1);
      }
    }
  }
}

template <int R, int W, int C, bool NT>
int run(const char *name, Ptrs &p, long n, int blocks) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((probe<R, W, C, NT>), dim3(blocks), dim3(256), 0, 0, p, n);
  CHECK(hipDeviceSynchronize());
  const int reps = 20;
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((probe<R, W, C, NT>), dim3(blocks), dim3(256), 0, 0, p, n);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double bytes = (double)(R + W) * n * 8.0;
  printf("%-28s R=%2d W=%2d C=%d nt=%d blocks=%6d  %8.3f ms  %7.1f GB/s\n", name, R, W, C, (int)NT,
         blocks, ms, bytes / (ms * 1e-3) / 1e9);
  return 0;
}

// The bench's step shape: CCLM (10 in / 7 out), MOM5 (11 / 7) and RCO (5 / 6) back to back on
// SHARED inputs, each writing its OWN outputs (as the three engines of bench.py do).  A kernel
// repeated on the same outputs can coalesce its writes with the previous launch's dirty lines
// in the memory-side Infinity Cache; in this sequence every launch writes fresh addresses.
int interleaved(const Ptrs &base, long n, int blocks) {
  Ptrs pc = base, pm = base, pr = base, pc2 = base;
  for (int w = 0; w < 7; ++w) pc.out[w] = base.out[w], pm.out[w] = base.out[7 + w], pc2.out[w] = base.out[7 + w];
  for (int w = 0; w < 6; ++w) pr.out[w] = base.out[14 + w];
  hipEvent_t ev[4];
  for (auto &h : ev) CHECK(hipEventCreate(&h));
  const int reps = 50;
  float t[3] = {0, 0, 0};
  for (int r = -5; r < reps; ++r) {
    CHECK(hipEventRecord(ev[0]));
    hipLaunchKernelGGL((probe<10, 7, 2, true>), dim3(blocks), dim3(256), 0, 0, pc, n);
    CHECK(hipEventRecord(ev[1]));
    hipLaunchKernelGGL((probe<11, 7, 2, true>), dim3(blocks), dim3(256), 0, 0, pm, n);
    CHECK(hipEventRecord(ev[2]));
    hipLaunchKernelGGL((probe<5, 6, 2, true>), dim3(blocks), dim3(256), 0, 0, pr, n);
    CHECK(hipEventRecord(ev[3]));
    CHECK(hipEventSynchronize(ev[3]));
    if (r < 0) continue;
    for (int k = 0; k < 3; ++k) {
      float ms;
      CHECK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
      t[k] += ms / reps;
    }
  }
  const int rw[3][2] = {{10, 7}, {11, 7}, {5, 6}};
  const char *nm[3] = {"interleaved cclm-shape nt", "interleaved mom5-shape nt", "interleaved rco-shape nt"};
  for (int k = 0; k < 3; ++k)
    printf("%-28s R=%2d W=%2d C=2 nt=1 blocks=%6d  %8.3f ms  %7.1f GB/s\n", nm[k], rw[k][0], rw[k][1], blocks, t[k],
           (rw[k][0] + rw[k][1]) * n * 8.0 / (t[k] * 1e-3) / 1e9);
  // one shape alternating between two output sets: fresh addresses every launch
  float alt = 0;
  for (int r = -4; r < 2 * reps; ++r) {
    CHECK(hipEventRecord(ev[0]));
    hipLaunchKernelGGL((probe<10, 7, 2, true>), dim3(blocks), dim3(256), 0, 0, (r & 1) ? pc2 : pc, n);
    CHECK(hipEventRecord(ev[1]));
    CHECK(hipEventSynchronize(ev[1]));
    float ms;
    CHECK(hipEventElapsedTime(&ms, ev[0], ev[1]));
    if (r >= 0) alt += ms / (2 * reps);
  }
  printf("%-28s R=%2d W=%2d C=2 nt=1 blocks=%6d  %8.3f ms  %7.1f GB/s\n", "cclm-shape nt, 2 out sets", 10, 7, blocks,
         alt, 17 * n * 8.0 / (alt * 1e-3) / 1e9);
  for (auto &h : ev) CHECK(hipEventDestroy(h));
  return 0;
}

int main() {
  // 10M cells x 8 B = 80 MB per array: a 17-array step (1.36 GB) is far beyond the 256 MB
  // Infinity Cache.  The 1-in/1-out copy uses 100M-element arrays (1.6 GB per launch) for
  // the same reason -- at 10M (160 MB) it would run from the Infinity Cache.
  const long n = 10'000'000, n_copy = 100'000'000;
  Ptrs p, pc;
  for (int i = 0; i < 32; ++i) {
    double *x;
    CHECK(hipMalloc(&x, n * sizeof(double)));
    CHECK(hipMemset(x, 0, n * sizeof(double)));
    p.in[i] = x;
    CHECK(hipMalloc(&p.out[i], n * sizeof(double)));
  }
  for (int i = 0; i < 32; ++i) pc.in[i] = nullptr, pc.out[i] = nullptr;
  {
    double *x, *y;
    CHECK(hipMalloc(&x, n_copy * sizeof(double)));
    CHECK(hipMemset(x, 0, n_copy * sizeof(double)));
    CHECK(hipMalloc(&y, n_copy * sizeof(double)));
    pc.in[0] = x;
    pc.out[0] = y;
  }
  for (int blocks : {2048, 8192, 0}) {
    run<1, 1, 2, false>("copy 1.6 GB", pc, n_copy, blocks ? blocks : (int)(n_copy / 2 / 256));
    run<1, 1, 2, true>("copy 1.6 GB nt", pc, n_copy, blocks ? blocks : (int)(n_copy / 2 / 256));
  }
  for (int blocks : {1024, 2048, 4096, 8192, 19532}) run<10, 7, 2, false>("cclm-shape", p, n, blocks);
  run<10, 7, 1, false>("cclm-shape", p, n, 2048);
  run<10, 7, 4, false>("cclm-shape", p, n, 2048);
  run<10, 7, 2, true>("cclm-shape", p, n, 2048);
  run<10, 7, 4, true>("cclm-shape", p, n, 2048);
  run<11, 7, 2, false>("mom5-shape", p, n, 2048);
  run<5, 6, 2, false>("rco-shape", p, n, 2048);
  run<16, 0, 2, false>("read-only 16", p, n, 2048);
  run<16, 0, 2, true>("read-only 16 nt", p, n, 2048);
  run<10, 7, 2, true>("cclm-shape nt", p, n, 8192);
  run<11, 7, 2, true>("mom5-shape nt", p, n, 8192);
  run<5, 6, 2, true>("rco-shape nt", p, n, 8192);
  // several surface types: T=2 CCLM (8 shared + 3 per type in, 7 per type + 7 averages out)
  // and T=6 with the accumulation-free shape, to see what many concurrent streams reach
  run<14, 21, 2, true>("T2 cclm-shape nt", p, n, 8192);
  run<26, 32, 2, true>("T4ish 26/32 nt", p, n, 8192);
  run<1, 16, 2, false>("write-heavy 1/16", p, n, 2048);
  if (interleaved(p, n, 8192)) return 1;
  return 0;
}
