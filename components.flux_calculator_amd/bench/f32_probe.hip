// f32_probe.hip -- the streaming ceiling of the fp32 engine's CCLM step shape (config 5):
// a tile-blocked read pool of 10 fp32 arrays and a write pool of 7 (4096-cell tiles), the map
// (int32 index + fp64 weight per cell) and six fp32 atmosphere outputs at a quarter of the
// cell rate; one 256-cell tile per wave (lane l: cells 4l..4l+3, 16-B loads and stores,
// non-temporal except the atmosphere stores, as in the product kernel), XCD runs of 16
// workgroups.  Trivial arithmetic, so the rate is what the memory system gives this shape.
// Layout 0: atmosphere runs line-aligned; 1: starting at arbitrary cells (random map).
// Several fresh allocation sets per layout, each at full occupancy and with 40 KB of dynamic
// LDS per workgroup (4 workgroups = 4 waves per SIMD, the product kernel's occupancy).
// Measurement only.
//   hipcc --offload-arch=gfx950 -O3 f32_probe.hip -o f32_probe && ./f32_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                                       \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));
constexpr long kTile = 4096;
constexpr int kR = 10, kW = 7, kA = 6;

struct Args {
  const float *rd;
  float *wr;
  const int *idx;
  const double *w;
  float *atm;
  long n;
};

__device__ __forceinline__ unsigned xcd_block(unsigned b, unsigned nb) {
  constexpr unsigned K = 16, row = K * 8;
  const unsigned full = nb / row * row;
  if (b >= full) return b;
  const unsigned x = b % 8, i = b / 8;
  return i / K * row + x * K + i % K;
}

template <int L>
__global__ __launch_bounds__(256) void step(Args a) {
  const long tile = (long)xcd_block(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long j = tile * 256 + 4 * lane;
  if (j >= a.n) return;
  const long t = j / kTile, o = j % kTile, row = t * kR * kTile;
  f4 s = {0, 0, 0, 0};
#pragma unroll
  for (int r = 0; r < kR; ++r) s += __builtin_nontemporal_load(reinterpret_cast<const f4 *>(a.rd + row + r * kTile + o));
  const i4 ii = *reinterpret_cast<const i4 *>(a.idx + j);
  const d2 w0 = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(a.w + j));
  const d2 w1 = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(a.w + j + 2));
  s.x = s.x * (float)w0[0] + ii.x;
  s.y = s.y * (float)w0[1] + ii.y;
  s.z = s.z * (float)w1[0] + ii.z;
  s.w = s.w * (float)w1[1] + ii.w;
#pragma unroll
  for (int k = 0; k < kW; ++k)
    __builtin_nontemporal_store(s * (float)(k + 1), reinterpret_cast<f4 *>(a.wr + row + k * kTile + o));
  const float q = s.x + s.y + s.z + s.w;
  long a0 = tile * 64, a1 = a0 + 64;
  if (L == 1) {
    auto off = [](long x) { return x == 0 ? 0L : (long)(((unsigned long)x * 2654435761ul >> 11) % 32) - 16; };
    a0 += off(tile);
    a1 += off(tile + 1);
  }
  if (lane < a1 - a0) {  // (runs of up to 80 values: lanes 0..63 take the first 64)
    const long av = a0 + lane, u = av / kTile, ao = av % kTile;
#pragma unroll
    for (int k = 0; k < kA; ++k) a.atm[(u * kA + k) * kTile + ao] = q * (k + 2);
  }
  if (lane + 64 < a1 - a0) {
    const long av = a0 + lane + 64, u = av / kTile, ao = av % kTile;
#pragma unroll
    for (int k = 0; k < kA; ++k) a.atm[(u * kA + k) * kTile + ao] = q * (k + 3);
  }
}

int main() {
  const long n = 10'000'000, tiles = (n + kTile - 1) / kTile;
  const long natm = n / 4 + 128, atiles = (natm + kTile - 1) / kTile + 1;
  const double alg = (kR + kW) * 4.0 + 12.0 + kA * 4.0 / 4.0;  // B/cell
  const int sets = 4, reps = 30;
  std::vector<double> mean[4];
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int blocks = (int)((n / 256 + 3) / 4);
  for (int set = 0; set < sets; ++set) {
    for (int LL : {0, 1, 2, 3}) {
      const int L = LL & 1;
      const size_t lds = LL >= 2 ? 40960 : 0;
      float *rd, *wr, *atm;
      int *idx;
      double *w;
      CHECK(hipMalloc(&rd, tiles * kR * kTile * 4));
      CHECK(hipMalloc(&wr, tiles * kR * kTile * 4));
      CHECK(hipMalloc(&atm, atiles * kA * kTile * 4));
      CHECK(hipMalloc(&idx, (n + 64) * 4));
      CHECK(hipMalloc(&w, (n + 64) * 8));
      CHECK(hipMemset(rd, 0, tiles * kR * kTile * 4));
      CHECK(hipMemset(idx, 0, (n + 64) * 4));
      CHECK(hipMemset(w, 0, (n + 64) * 8));
      Args a{rd, wr, idx, w, atm, n};
      auto launch = [&]() {
        if (L == 0) hipLaunchKernelGGL(step<0>, dim3(blocks), dim3(256), lds, 0, a);
        else hipLaunchKernelGGL(step<1>, dim3(blocks), dim3(256), lds, 0, a);
      };
      for (int i = 0; i < 300; ++i) launch();
      std::vector<float> ms(reps);
      for (int i = 0; i < reps; ++i) {
        CHECK(hipEventRecord(e0));
        launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms[i], e0, e1));
      }
      CHECK(hipGetLastError());
      double m = 0;
      for (float x : ms) m += x;
      m /= reps;
      mean[LL].push_back(alg * n / (m * 1e-3) / 1e9);
      printf("set %d layout %d lds %zu: mean %.1f GB/s (%.4f ms)\n", set, L, lds, mean[LL].back(), m);
      fflush(stdout);
      CHECK(hipFree(rd));
      CHECK(hipFree(wr));
      CHECK(hipFree(atm));
      CHECK(hipFree(idx));
      CHECK(hipFree(w));
    }
  }
  const char *names[4] = {"aligned atmosphere runs", "atmosphere runs at arbitrary cells",
                          "aligned, 4 waves per SIMD", "arbitrary, 4 waves per SIMD"};
  for (int L = 0; L < 4; ++L) {
    double m = 0;
    for (double x : mean[L]) m += x;
    printf("layout %d (%s): mean over %d sets %.1f GB/s\n", L, names[L], sets, m / sets);
  }
  return 0;
}
