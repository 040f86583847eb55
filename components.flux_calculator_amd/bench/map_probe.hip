// map_probe.hip -- where should the exchange->atmosphere map (int32 index + fp64 weight per
// exchange cell) live relative to the tile-blocked field pools?  The CCLM fused step's access
// shape with trivial arithmetic: a read pool of 10 fp64 arrays and a write pool of 7 (tiles of
// 4096 cells, S slots per tile row), the map (12 B/cell), and six atmosphere outputs at a
// quarter of the cell rate in a tile-blocked atmosphere pool; one 128-cell tile per wave, lane
// l cells 2l and 2l+1, non-temporal 16-B loads and stores, XCD runs of 64 workgroups as in
// the product kernels.  Layouts of the map:
//   0 separate: idx and w contiguous arrays of their own (libfcx today)
//   1 in the read pool: idx and w two more slots of every read tile row (S = 12)
//   2 map pool: [tile][4096 idx][4096 w] in one allocation of its own
//   3 as 0, but every wave's atmosphere range starts at an arbitrary cell (32 t + a fixed
//     pseudo-random offset in [-8, 8)), as on the random map: its stores begin and end
//     inside 128-B lines that the neighbouring waves also write
//   4 as 3 with plain (temporal) atmosphere stores
//   5 as 3, the block's four waves' atmosphere values staged in LDS and stored by the block
//     after a barrier, so only the lines at the block's two ends are shared with other
//     workgroups
// Every layout is measured on several fresh allocation sets (physical placement moves a
// many-stream kernel by several per cent) in an interleaved order.  Measurement only.
//   hipcc --offload-arch=gfx950 -O3 map_probe.hip -o map_probe && ./map_probe
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

typedef double d2 __attribute__((ext_vector_type(2)));
typedef int i2 __attribute__((ext_vector_type(2)));
constexpr long kTile = 4096;  // layout tile (cells)
constexpr int kR = 10, kW = 7, kA = 6;

struct Args {
  const double *rd;  // read pool base (slot k of tile row t at (t * S + k) * kTile)
  double *wr;        // write pool base
  const int *idx;    // layout 0: contiguous; 1: read-pool slot kR (int view); 2: map pool
  const double *w;   // layout 0: contiguous; 1: read-pool slot kR + 1; 2: map pool
  double *atm;       // atmosphere pool: field k of atm tile u at (u * kA + k) * kTile
  long S;            // slots per field tile row
  long n;
};

__device__ __forceinline__ unsigned xcd_block(unsigned b, unsigned nb) {
  constexpr unsigned K = 64, row = K * 8;
  const unsigned full = nb / row * row;
  if (b >= full) return b;
  const unsigned x = b % 8, i = b / 8;
  return i / K * row + x * K + i % K;
}

template <int L>
__global__ __launch_bounds__(256) void step(Args a) {
  const long tile = (long)xcd_block(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long jj = tile * 128 + 2 * lane;
  if (L != 5 && jj >= a.n) return;
  const bool live = jj < a.n;  // (L = 5: every wave reaches the block barrier)
  const long j = live ? jj : 0;
  const long t = j / kTile, o = j % kTile;
  const long row = t * a.S * kTile;
  double s0 = 0, s1 = 0;
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(a.rd + row + r * kTile + o));
    s0 += v[0];
    s1 += v[1];
  }
  i2 ii;
  d2 ww;
  if (L == 0 || L >= 3) {
    ii = *reinterpret_cast<const i2 *>(a.idx + j);
    ww = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(a.w + j));
  } else if (L == 1) {
    ii = *reinterpret_cast<const i2 *>(reinterpret_cast<const int *>(a.rd + row + kR * kTile) + o);
    ww = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(a.rd + row + (kR + 1) * kTile + o));
  } else {
    const char *m = reinterpret_cast<const char *>(a.idx) + t * kTile * 12;
    ii = *reinterpret_cast<const i2 *>(reinterpret_cast<const int *>(m) + o);
    ww = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(reinterpret_cast<const double *>(m + kTile * 4) + o));
  }
  s0 = s0 * ww[0] + ii[0];
  s1 = s1 * ww[1] + ii[1];
#pragma unroll
  for (int k = 0; k < kW; ++k)
    if (live) __builtin_nontemporal_store(d2{s0 * (k + 1), s1 * (k + 1)}, reinterpret_cast<d2 *>(a.wr + row + k * kTile + o));
  // a quarter of the cell rate: lanes 0..31 store the wave's 32 atmosphere values per field
  const double q = __shfl_xor(s0 + s1, 1);
  long a0 = tile * 32, a1 = a0 + 32;
  if (L >= 3) {
    auto off = [](long x) { return x == 0 ? 0L : (long)(((unsigned long)x * 2654435761ul >> 11) % 16) - 8; };
    a0 += off(tile);
    a1 += off(tile + 1);
  }
  if (L == 5) {  // block staging: [field][up to 4 x 40 values] in LDS
    __shared__ double st[kA][4 * 40];
    __shared__ long lo_hi[2];
    const int wv = threadIdx.x >> 6;
    auto off = [](long x) { return x == 0 ? 0L : (long)(((unsigned long)x * 2654435761ul >> 11) % 16) - 8; };
    const long tb = tile - wv;  // the block's first tile
    const long b0 = tb * 32 + off(tb), b1 = (tb + 4) * 32 + off(tb + 4);
    if (live && lane < a1 - a0)
      for (int k = 0; k < kA; ++k) st[k][a0 - b0 + lane] = q * (k + 2);
    __syncthreads();
    const long b1c = min(b1, (a.n / 128) * 32);  // (the grid's last block: its live waves only)
    for (long i = threadIdx.x; i < b1c - b0; i += 256) {
      const long av = b0 + i, u = av / kTile, ao = av % kTile;
#pragma unroll
      for (int k = 0; k < kA; ++k) __builtin_nontemporal_store(st[k][i], a.atm + (u * kA + k) * kTile + ao);
    }
    (void)lo_hi;
    return;
  }
  if (lane < a1 - a0) {
    const long av = a0 + lane, u = av / kTile, ao = av % kTile;
#pragma unroll
    for (int k = 0; k < kA; ++k) {
      if (L == 4) a.atm[(u * kA + k) * kTile + ao] = q * (k + 2);
      else __builtin_nontemporal_store(q * (k + 2), a.atm + (u * kA + k) * kTile + ao);
    }
  }
}

int main() {
  const long n = 10'000'000, tiles = (n + kTile - 1) / kTile;
  const long natm = n / 4 + 64, atiles = (natm + kTile - 1) / kTile + 1;
  const double alg = (kR + kW) * 8.0 + 12.0 + kA * 8.0 / 4.0;  // B/cell
  const int sets = 4, reps = 30;
  std::vector<double> best[6], mean[6];
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int blocks = (int)((n / 128 + 3) / 4);
  for (int set = 0; set < sets; ++set) {
    for (int L : {0, 3, 4, 5}) {
      const long S = L == 1 ? kR + 2 : kR;
      double *rd, *wr, *atm, *w = nullptr;
      int *idx = nullptr;
      CHECK(hipMalloc(&rd, tiles * S * kTile * 8));
      CHECK(hipMalloc(&wr, tiles * S * kTile * 8));
      CHECK(hipMalloc(&atm, atiles * kA * kTile * 8));
      if (L == 0 || L >= 3) {
        CHECK(hipMalloc(&idx, n * 4));
        CHECK(hipMalloc(&w, n * 8));
      } else if (L == 2) {
        CHECK(hipMalloc(&idx, tiles * kTile * 12));
        w = reinterpret_cast<double *>(idx);
      }
      CHECK(hipMemset(rd, 0, tiles * S * kTile * 8));
      if (L != 1) CHECK(hipMemset(idx, 0, L == 2 ? tiles * kTile * 12 : n * 4));
      if (L == 0 || L >= 3) CHECK(hipMemset(w, 0, n * 8));
      Args a{rd, wr, idx, w, atm, S, n};
      auto launch = [&]() {
        if (L == 0) hipLaunchKernelGGL(step<0>, dim3(blocks), dim3(256), 0, 0, a);
        else if (L == 1) hipLaunchKernelGGL(step<1>, dim3(blocks), dim3(256), 0, 0, a);
        else if (L == 3) hipLaunchKernelGGL(step<3>, dim3(blocks), dim3(256), 0, 0, a);
        else if (L == 4) hipLaunchKernelGGL(step<4>, dim3(blocks), dim3(256), 0, 0, a);
        else if (L == 5) hipLaunchKernelGGL(step<5>, dim3(blocks), dim3(256), 0, 0, a);
        else hipLaunchKernelGGL(step<2>, dim3(blocks), dim3(256), 0, 0, a);
      };
      for (int i = 0; i < 200; ++i) launch();  // clocks up
      std::vector<float> ms(reps);
      for (int i = 0; i < reps; ++i) {
        CHECK(hipEventRecord(e0));
        launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms[i], e0, e1));
      }
      CHECK(hipGetLastError());
      std::sort(ms.begin(), ms.end());
      double m = 0;
      for (float x : ms) m += x;
      m /= reps;
      best[L].push_back(alg * n / (ms[0] * 1e-3) / 1e9);
      mean[L].push_back(alg * n / (m * 1e-3) / 1e9);
      printf("set %d layout %d: mean %.1f GB/s, best %.1f GB/s\n", set, L, mean[L].back(), best[L].back());
      fflush(stdout);
      CHECK(hipFree(rd));
      CHECK(hipFree(wr));
      CHECK(hipFree(atm));
      if (idx) CHECK(hipFree(idx));
      if (L == 0 || L >= 3) CHECK(hipFree(w));
    }
  }
  const char *names[6] = {"separate", "in read pool", "map pool", "atmosphere ranges misaligned",
                          "misaligned, temporal atmosphere stores", "misaligned, block-staged atmosphere stores"};
  for (int L : {0, 3, 4, 5}) {
    double m = 0;
    for (double x : mean[L]) m += x;
    printf("layout %d (%s): mean over %d sets %.1f GB/s\n", L, names[L], sets, m / sets);
  }
  return 0;
}
