// glds_probe.hip -- do LDS-DMA loads (global_load_lds_dwordx4) stream the flux kernel's
// many-array pattern faster than register loads?  CCLM shape (10 fp64 inputs, 7 outputs),
// 10M cells, one 128-cell tile per wave, full grid, non-temporal; both kernels hold the same
// LDS per block, so they run at the same occupancy (4 blocks of 4 waves per CU).  Output sets
// rotate so no launch rewrites the previous launch's lines.  Measurement tool only.
//   hipcc --offload-arch=gfx950 -O3 glds_probe.hip -o glds_probe && ./glds_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) {                                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                                        \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;
constexpr int R = 10, W = 7, kTile = 128;

struct Ptrs {
  const double *in[R];
  double *out[W];
};

// MODE 0: register loads; 1: LDS-DMA loads then ds_read; 2: register loads, no LDS held
template <int MODE>
__global__ __launch_bounds__(256) void probe(Ptrs p, long n) {
  __shared__ double s[MODE == 2 ? 1 : 4 * R * kTile];  // 40 KB per block in modes 0 and 1
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long t0 = ((long)blockIdx.x * 4 + wv) * kTile;
  if (t0 >= n) return;
  const long j = t0 + 2 * lane;
  double a0 = 0.0, a1 = 0.0;
  if constexpr (MODE == 1) {
    double *mine = s + wv * R * kTile;
#pragma unroll
    for (int r = 0; r < R; ++r)
      __builtin_amdgcn_global_load_lds((const void *)(p.in[r] + j), (lds_void *)(mine + r * kTile), 16, 0, 2);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const d2 t = *reinterpret_cast<const d2 *>(mine + r * kTile + 2 * lane);
      a0 += t[0];
      a1 += t[1];
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const d2 t = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(p.in[r] + j));
      a0 += t[0];
      a1 += t[1];
    }
    if constexpr (MODE == 0) {
      if (a0 == 1234.5) s[threadIdx.x] = a1;  // keep the LDS allocation (occupancy) alive
    }
  }
#pragma unroll
  for (int w = 0; w < W; ++w)
    __builtin_nontemporal_store(d2{a0 * (w + 1), a1 * (w + 1)}, reinterpret_cast<d2 *>(p.out[w] + j));
}

template <int MODE>
float run(Ptrs *sets, long n, int reps) {
  const int blocks = (int)((n / kTile + 3) / 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 6; ++i) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, sets[i % 3], n);
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, sets[i % 3], n);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps;
}

int main() {
  const long n = 10'000'000;  // multiple of 128
  Ptrs sets[3];
  double *in[R];
  for (int r = 0; r < R; ++r) {
    CHECK(hipMalloc(&in[r], n * sizeof(double)));
    CHECK(hipMemset(in[r], 0, n * sizeof(double)));
  }
  for (int k = 0; k < 3; ++k) {
    for (int r = 0; r < R; ++r) sets[k].in[r] = in[r];
    for (int w = 0; w < W; ++w) CHECK(hipMalloc(&sets[k].out[w], n * sizeof(double)));
  }
  const double bytes = (R + W) * n * 8.0;
  for (int round = 0; round < 4; ++round) {
    const float m0 = run<0>(sets, n, 30), m1 = run<1>(sets, n, 30), m2 = run<2>(sets, n, 30);
    printf("round %d  registers (4 blk/CU) %7.1f GB/s   LDS-DMA (4 blk/CU) %7.1f GB/s   registers (no LDS) %7.1f GB/s\n",
           round, bytes / (m0 * 1e6), bytes / (m1 * 1e6), bytes / (m2 * 1e6));
  }
  return 0;
}
