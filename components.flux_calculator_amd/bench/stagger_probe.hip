// stagger_probe.hip -- does the placement of the 17 SoA streams of a fused flux launch move
// the HBM ceiling?  Same trivial-arithmetic kernel shape as stream_probe.hip (CCLM: 10 in,
// 7 out, fp64, 2 cells per lane, non-temporal), with the arrays carved out of one pool at
// base_k = k * (array bytes rounded to 2 MiB) + k * S for a stagger S, against separate
// hipMallocs.  Measurement tool only, not part of the product.
//   hipcc --offload-arch=gfx950 -O3 stagger_probe.hip -o stagger_probe && ./stagger_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <initializer_list>

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
  const double *in[16];
  double *out[16];
};

template <int R, int W>
__global__ __launch_bounds__(256) void probe(Ptrs p, long n) {
  const long units = n / 2;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long u = (long)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += stride) {
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      d2 t = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(p.in[r]) + u);
      a0 += t[0];
      a1 += t[1];
    }
#pragma unroll
    for (int w = 0; w < W; ++w)
      __builtin_nontemporal_store(d2{a0 * (w + 1), a1 * (w + 1)}, reinterpret_cast<d2 *>(p.out[w]) + u);
  }
}

// three shapes back to back like the bench step; each writes its own outputs
template <int R, int W>
float time_shape(const Ptrs &p, long n, int blocks, hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  for (int r = -5; r < 40; ++r) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((probe<R, W>), dim3(blocks), dim3(256), 0, 0, p, n);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float t;
    (void)hipEventElapsedTime(&t, a, b);
    if (r >= 0) ms += t / 40;
  }
  return ms;
}

int measure(const char *label, double *const *arr, long n) {
  // arr[0..10] inputs (shared), arr[11..17] CCLM out, arr[18..24] MOM5 out, arr[25..30] RCO out
  Ptrs pc{}, pm{}, pr{};
  for (int i = 0; i < 11; ++i) pc.in[i] = pm.in[i] = pr.in[i] = arr[i];
  for (int w = 0; w < 7; ++w) pc.out[w] = arr[11 + w], pm.out[w] = arr[18 + w];
  for (int w = 0; w < 6; ++w) pr.out[w] = arr[25 + w];
  hipEvent_t ev[4];
  for (auto &h : ev) CHECK(hipEventCreate(&h));
  for (int blocks : {8192, (int)(n / 2 / 256)}) {
    const int reps = 50;
    float t[3] = {0, 0, 0};
    for (int r = -10; r < reps; ++r) {
      (void)hipEventRecord(ev[0]);
      hipLaunchKernelGGL((probe<10, 7>), dim3(blocks), dim3(256), 0, 0, pc, n);
      (void)hipEventRecord(ev[1]);
      hipLaunchKernelGGL((probe<11, 7>), dim3(blocks), dim3(256), 0, 0, pm, n);
      (void)hipEventRecord(ev[2]);
      hipLaunchKernelGGL((probe<5, 6>), dim3(blocks), dim3(256), 0, 0, pr, n);
      (void)hipEventRecord(ev[3]);
      CHECK(hipEventSynchronize(ev[3]));
      if (r < 0) continue;
      for (int k = 0; k < 3; ++k) {
        float ms;
        (void)hipEventElapsedTime(&ms, ev[k], ev[k + 1]);
        t[k] += ms / reps;
      }
    }
    const int rw[3] = {17, 18, 11};
    printf("%-34s blocks=%6d  cclm %6.1f  mom5 %6.1f  rco %6.1f GB/s  (step %.3f ms)\n", label, blocks,
           rw[0] * n * 8.0 / (t[0] * 1e6), rw[1] * n * 8.0 / (t[1] * 1e6), rw[2] * n * 8.0 / (t[2] * 1e6),
           t[0] + t[1] + t[2]);
  }
  for (auto &h : ev) CHECK(hipEventDestroy(h));
  return 0;
}

int main(int argc, char **argv) {
  const long n = 10'000'000;
  const size_t bytes = n * sizeof(double);
  const size_t two_mb = 2u << 20;
  const int A = 31;
  const int rounds = argc > 1 ? atoi(argv[1]) : 1;
  if (argc > 2 && !strcmp(argv[2], "alloc")) {  // fresh sets of separate allocations
    for (int set = 0; set < rounds; ++set) {
      double *arr[A];
      void *pad = nullptr;
      if (set % 2) CHECK(hipMalloc(&pad, (size_t)(set * 37 + 1) << 20));  // shift the next VAs
      for (int i = 0; i < A; ++i) {
        CHECK(hipMalloc(&arr[i], bytes));
        CHECK(hipMemset(arr[i], 0, bytes));
      }
      printf("set %d: VA of array 0 %p, deltas (MiB):", set, (void *)arr[0]);
      for (int i = 1; i < 6; ++i) printf(" %.2f", ((char *)arr[i] - (char *)arr[i - 1]) / 1048576.0);
      printf("\n");
      char label[64];
      snprintf(label, sizeof label, "separate, set %d", set);
      if (measure(label, arr, n)) return 1;
      for (int i = 0; i < A; ++i) CHECK(hipFree(arr[i]));
      if (pad) CHECK(hipFree(pad));
    }
    return 0;
  }
  double *sep[A];
  for (int i = 0; i < A; ++i) {
    CHECK(hipMalloc(&sep[i], bytes));
    CHECK(hipMemset(sep[i], 0, bytes));
  }
  const size_t rounded = (bytes + two_mb - 1) / two_mb * two_mb;
  char *pool;
  const size_t pool_bytes = A * (rounded + (4u << 20)) + (8u << 20);
  CHECK(hipMalloc(&pool, pool_bytes));
  CHECK(hipMemset(pool, 0, pool_bytes));
  const size_t staggers[] = {0, 256, 1024, 4096, 8192, 65536, 2u << 20, 4352, 3u << 20};
  for (int r = 0; r < rounds; ++r) {
    if (measure("separate hipMalloc", sep, n)) return 1;
    for (size_t s : (rounds > 1 ? std::initializer_list<size_t>{0, 65536} : std::initializer_list<size_t>{0, 256, 1024, 4096, 8192, 65536, 2u << 20, 4352, 3u << 20})) {
      double *arr[A];
      for (int i = 0; i < A; ++i) arr[i] = reinterpret_cast<double *>(pool + i * rounded + i * s);
      char label[64];
      snprintf(label, sizeof label, "pool, stagger %zu B", s);
      if (measure(label, arr, n)) return 1;
    }
  }
  (void)staggers;
  if (rounds == 1) {  // power-of-two strides: 128 MiB apart (worst case for address bits alike)
    char *pool2;
    const size_t p2 = size_t(128) << 20;
    CHECK(hipMalloc(&pool2, A * p2));
    double *arr[A];
    for (int i = 0; i < A; ++i) arr[i] = reinterpret_cast<double *>(pool2 + i * p2);
    if (measure("pool, 128 MiB apart", arr, n)) return 1;
    for (int i = 0; i < A; ++i) arr[i] = reinterpret_cast<double *>(pool2 + i * p2 + i * 4096);
    if (measure("pool, 128 MiB apart + 4 KiB*k", arr, n)) return 1;
    CHECK(hipFree(pool2));
  }
  CHECK(hipFree(pool));
  for (int i = 0; i < A; ++i) CHECK(hipFree(sep[i]));
  return 0;
}
