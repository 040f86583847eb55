// layout_probe.hip -- does a tile-blocked device layout (AoSoA: [tile][var][TILE cells])
// stream faster than the struct-of-arrays mirrors (one array per variable) on MI355X?
// Same access shape as the fused flux kernels (CCLM 10 in / 7 out, MOM5 11 / 7, RCO 5 / 6),
// trivial arithmetic, non-temporal 16-B loads and stores, one trip per wave (a wave owns 128
// cells, lane l cells 2l and 2l+1).  Measurement only, not part of the product.
//   hipcc --offload-arch=gfx950 -O3 layout_probe.hip -o layout_probe && ./layout_probe
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
constexpr int kWaveCells = 128;

struct Ptrs {
  const double *in[16];
  double *out[16];
};

// SoA: in[r][cell], out[w][cell]
template <int R, int W>
__global__ __launch_bounds__(256) void soa(Ptrs p, long n) {
  const long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long j = t * kWaveCells + 2 * (threadIdx.x & 63);
  if (j >= n) return;
  double a0 = 0, a1 = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(p.in[r] + j));
    a0 += v[0];
    a1 += v[1];
  }
#pragma unroll
  for (int w = 0; w < W; ++w)
    __builtin_nontemporal_store(d2{a0 * (w + 1), a1 * (w + 1)}, reinterpret_cast<d2 *>(p.out[w] + j));
}

// SoA, each wave walking K consecutive 128-cell tiles (a contiguous run of K KiB per array)
template <int R, int W, int K>
__global__ __launch_bounds__(256) void soa_run(Ptrs p, long n) {
  const long w0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * K;
  for (int k = 0; k < K; ++k) {
    const long j = (w0 + k) * kWaveCells + 2 * (threadIdx.x & 63);
    if (j >= n) return;
    double a0 = 0, a1 = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(p.in[r] + j));
      a0 += v[0];
      a1 += v[1];
    }
#pragma unroll
    for (int w = 0; w < W; ++w)
      __builtin_nontemporal_store(d2{a0 * (w + 1), a1 * (w + 1)}, reinterpret_cast<d2 *>(p.out[w] + j));
  }
}

// SoA, block-contiguous runs: the 4 waves of a block take 4 adjacent tiles, the block walks
// K such groups (512*K contiguous cells per block)
template <int R, int W, int K>
__global__ __launch_bounds__(256) void soa_brun(Ptrs p, long n) {
  for (int k = 0; k < K; ++k) {
    const long t = ((long)blockIdx.x * K + k) * 4 + (threadIdx.x >> 6);
    const long j = t * kWaveCells + 2 * (threadIdx.x & 63);
    if (j >= n) return;
    double a0 = 0, a1 = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(p.in[r] + j));
      a0 += v[0];
      a1 += v[1];
    }
#pragma unroll
    for (int w = 0; w < W; ++w)
      __builtin_nontemporal_store(d2{a0 * (w + 1), a1 * (w + 1)}, reinterpret_cast<d2 *>(p.out[w] + j));
  }
}

// AoSoA: block b of TILE cells holds var r at in[b*R*TILE + r*TILE + (cell % TILE)]
template <int R, int W, int TILE>
__global__ __launch_bounds__(256) void aosoa(const double *__restrict__ in, double *__restrict__ out, long n) {
  const long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long j = t * kWaveCells + 2 * (threadIdx.x & 63);
  if (j >= n) return;
  const long b = j / TILE, o = j % TILE;
  const double *ib = in + b * (long)R * TILE + o;
  double *ob = out + b * (long)W * TILE + o;
  double a0 = 0, a1 = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(ib + r * TILE));
    a0 += v[0];
    a1 += v[1];
  }
#pragma unroll
  for (int w = 0; w < W; ++w)
    __builtin_nontemporal_store(d2{a0 * (w + 1), a1 * (w + 1)}, reinterpret_cast<d2 *>(ob + w * TILE));
}

// one pool per kernel holding inputs AND outputs: block b of TILE cells, V slots; the
// kernel reads slots [s0, s0+R) and writes [s0+R, s0+R+W) (V > R+W: a subset of the pool)
template <int R, int W, int TILE>
__global__ __launch_bounds__(256) void pool(double *__restrict__ p, long n, int V, int s0) {
  const long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long j = t * kWaveCells + 2 * (threadIdx.x & 63);
  if (j >= n) return;
  const long b = j / TILE, o = j % TILE;
  double *pb = p + b * (long)V * TILE + (long)s0 * TILE + o;
  double a0 = 0, a1 = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(pb + r * TILE));
    a0 += v[0];
    a1 += v[1];
  }
#pragma unroll
  for (int w = 0; w < W; ++w)
    __builtin_nontemporal_store(d2{a0 * (w + 1), a1 * (w + 1)}, reinterpret_cast<d2 *>(pb + (R + w) * TILE));
}

// AoSoA with one stride S (slots) for both pools: the smaller pool has unused slots
template <int R, int W, int TILE>
__global__ __launch_bounds__(256) void aosoa_s(const double *__restrict__ in, double *__restrict__ out, long n, int S) {
  const long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long j = t * kWaveCells + 2 * (threadIdx.x & 63);
  if (j >= n) return;
  const long b = j / TILE, o = j % TILE;
  const double *ib = in + b * (long)S * TILE + o;
  double *ob = out + b * (long)S * TILE + o;
  double a0 = 0, a1 = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(ib + r * TILE));
    a0 += v[0];
    a1 += v[1];
  }
#pragma unroll
  for (int w = 0; w < W; ++w)
    __builtin_nontemporal_store(d2{a0 * (w + 1), a1 * (w + 1)}, reinterpret_cast<d2 *>(ob + w * TILE));
}

// the bench's step: three shapes back to back, own inputs and outputs each; returns per-kernel ms
template <class L0, class L1, class L2>
int step3(const char *name, L0 l0, L1 l1, L2 l2, long n) {
  hipEvent_t ev[4];
  for (auto &h : ev) CHECK(hipEventCreate(&h));
  const int reps = 100;
  float t[3] = {0, 0, 0};
  for (int r = -100; r < reps; ++r) {
    CHECK(hipEventRecord(ev[0]));
    l0();
    CHECK(hipEventRecord(ev[1]));
    l1();
    CHECK(hipEventRecord(ev[2]));
    l2();
    CHECK(hipEventRecord(ev[3]));
    CHECK(hipEventSynchronize(ev[3]));
    if (r < 0) continue;
    for (int k = 0; k < 3; ++k) {
      float ms;
      CHECK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
      t[k] += ms / reps;
    }
  }
  const int rw[3] = {17, 18, 11};
  double tot_b = 0, tot_t = 0;
  printf("%-22s", name);
  for (int k = 0; k < 3; ++k) {
    printf("  %6.3f ms %7.1f GB/s", t[k], rw[k] * n * 8.0 / (t[k] * 1e-3) / 1e9);
    tot_b += rw[k] * n * 8.0;
    tot_t += t[k];
  }
  printf("  | step %6.3f ms %7.1f GB/s\n", tot_t, tot_b / (tot_t * 1e-3) / 1e9);
  for (auto &h : ev) CHECK(hipEventDestroy(h));
  return 0;
}

template <int K>
int run_soa_run(long n, Ptrs *p) {
  const int blocks = (int)((n / kWaveCells / K + 3) / 4 + 1);
  char name[64];
  snprintf(name, sizeof name, "soa wave-run %d", K);
  if (step3(
          name, [&] { hipLaunchKernelGGL((soa_run<10, 7, K>), dim3(blocks), dim3(256), 0, 0, p[0], n); },
          [&] { hipLaunchKernelGGL((soa_run<11, 7, K>), dim3(blocks), dim3(256), 0, 0, p[1], n); },
          [&] { hipLaunchKernelGGL((soa_run<5, 6, K>), dim3(blocks), dim3(256), 0, 0, p[2], n); }, n))
    return 1;
  snprintf(name, sizeof name, "soa block-run %d", K);
  return step3(
      name, [&] { hipLaunchKernelGGL((soa_brun<10, 7, K>), dim3(blocks), dim3(256), 0, 0, p[0], n); },
      [&] { hipLaunchKernelGGL((soa_brun<11, 7, K>), dim3(blocks), dim3(256), 0, 0, p[1], n); },
      [&] { hipLaunchKernelGGL((soa_brun<5, 6, K>), dim3(blocks), dim3(256), 0, 0, p[2], n); }, n);
}

template <int TILE>
int run_aosoa(long n, double *ib[3], double *ob[3]) {
  const int blocks = (int)((n / kWaveCells + 3) / 4);
  char name[64];
  snprintf(name, sizeof name, "aosoa tile %d", TILE);
  return step3(
      name, [&] { hipLaunchKernelGGL((aosoa<10, 7, TILE>), dim3(blocks), dim3(256), 0, 0, ib[0], ob[0], n); },
      [&] { hipLaunchKernelGGL((aosoa<11, 7, TILE>), dim3(blocks), dim3(256), 0, 0, ib[1], ob[1], n); },
      [&] { hipLaunchKernelGGL((aosoa<5, 6, TILE>), dim3(blocks), dim3(256), 0, 0, ib[2], ob[2], n); }, n);
}

template <int TILE>
int run_pool(long n, double *pp[3], double *big) {
  const int blocks = (int)((n / kWaveCells + 3) / 4);
  char name[64];
  snprintf(name, sizeof name, "pool17 tile %d", TILE);
  if (step3(
          name, [&] { hipLaunchKernelGGL((pool<10, 7, TILE>), dim3(blocks), dim3(256), 0, 0, pp[0], n, 17, 0); },
          [&] { hipLaunchKernelGGL((pool<11, 7, TILE>), dim3(blocks), dim3(256), 0, 0, pp[1], n, 18, 0); },
          [&] { hipLaunchKernelGGL((pool<5, 6, TILE>), dim3(blocks), dim3(256), 0, 0, pp[2], n, 11, 0); }, n))
    return 1;
  // one shared pool of 46 slots for all three (each kernel touches its own 17/18/11)
  snprintf(name, sizeof name, "pool46 tile %d", TILE);
  return step3(
      name, [&] { hipLaunchKernelGGL((pool<10, 7, TILE>), dim3(blocks), dim3(256), 0, 0, big, n, 46, 0); },
      [&] { hipLaunchKernelGGL((pool<11, 7, TILE>), dim3(blocks), dim3(256), 0, 0, big, n, 46, 17); },
      [&] { hipLaunchKernelGGL((pool<5, 6, TILE>), dim3(blocks), dim3(256), 0, 0, big, n, 46, 35); }, n);
}

template <int TILE>
int run_s(long n, double *ib[3], double *ob[3]) {
  const int blocks = (int)((n / kWaveCells + 3) / 4);
  char name[64];
  snprintf(name, sizeof name, "aosoa 1-stride %d", TILE);
  return step3(
      name, [&] { hipLaunchKernelGGL((aosoa_s<10, 7, TILE>), dim3(blocks), dim3(256), 0, 0, ib[0], ob[0], n, 10); },
      [&] { hipLaunchKernelGGL((aosoa_s<11, 7, TILE>), dim3(blocks), dim3(256), 0, 0, ib[1], ob[1], n, 11); },
      [&] { hipLaunchKernelGGL((aosoa_s<5, 6, TILE>), dim3(blocks), dim3(256), 0, 0, ib[2], ob[2], n, 6); }, n);
}

int main() {
  const long n = 10'000'000;  // multiple of 1024 cells not required: tiles past n are skipped
  const int R[3] = {10, 11, 5}, W[3] = {7, 7, 6};
  Ptrs p[3];
  double *ib[3], *ob[3];
  for (int k = 0; k < 3; ++k) {
    for (int r = 0; r < R[k]; ++r) {
      double *x;
      CHECK(hipMalloc(&x, n * sizeof(double)));
      CHECK(hipMemset(x, 0, n * sizeof(double)));
      p[k].in[r] = x;
    }
    for (int w = 0; w < W[k]; ++w) CHECK(hipMalloc(&p[k].out[w], n * sizeof(double)));
  }
  const long np = (n + 262143) / 262144 * 262144;  // padded to whole tiles of any size probed
  for (int k = 0; k < 3; ++k) {
    CHECK(hipMalloc(&ib[k], np * 11 * sizeof(double)));
    CHECK(hipMemset(ib[k], 0, np * 11 * sizeof(double)));
    CHECK(hipMalloc(&ob[k], np * 11 * sizeof(double)));
  }
  double *pp[3], *big;
  for (int k = 0; k < 3; ++k) {
    CHECK(hipMalloc(&pp[k], np * (R[k] + W[k]) * sizeof(double)));
    CHECK(hipMemset(pp[k], 0, np * (R[k] + W[k]) * sizeof(double)));
  }
  CHECK(hipMalloc(&big, np * 46 * sizeof(double)));
  CHECK(hipMemset(big, 0, np * 46 * sizeof(double)));
  const int blocks = (int)((n / kWaveCells + 3) / 4);
  for (int rep = 0; rep < 2; ++rep) {
    if (step3(
            "soa", [&] { hipLaunchKernelGGL((soa<10, 7>), dim3(blocks), dim3(256), 0, 0, p[0], n); },
            [&] { hipLaunchKernelGGL((soa<11, 7>), dim3(blocks), dim3(256), 0, 0, p[1], n); },
            [&] { hipLaunchKernelGGL((soa<5, 6>), dim3(blocks), dim3(256), 0, 0, p[2], n); }, n))
      return 1;
    if (run_aosoa<2048>(n, ib, ob) || run_aosoa<4096>(n, ib, ob) || run_aosoa<8192>(n, ib, ob))
      return 1;
    if (run_s<4096>(n, ib, ob) || run_s<2048>(n, ib, ob)) return 1;
  }
  return 0;
}
