// Stress test of fcx::CopyPool (components.flux_calculator_amd/csrc/fcx_copy_pool.h), the
// host copy threads of the staging arena: many batches of random size and thread count,
// back to back and after idle gaps (workers asleep), each checked byte for byte.  An alarm
// turns a hang (a worker that misses a batch) into a failure.
#include <unistd.h>

#include <cstdio>
#include <random>

#include "fcx_copy_pool.h"

int main(int argc, char **argv) {
  alarm(120);
  const int batches = argc > 1 ? std::atoi(argv[1]) : 20000;
  std::mt19937 rng(12345);
  std::vector<char> src(1 << 20), dst(1 << 20);
  for (size_t i = 0; i < src.size(); ++i) src[i] = (char)rng();
  for (int b = 0; b < batches; ++b) {
    const int threads = 1 + (int)(rng() % 9);
    const int njobs = (int)(rng() % 40);
    std::vector<fcx::CopyJob> jobs;
    std::fill(dst.begin(), dst.end(), 0);
    size_t off = 0;
    for (int j = 0; j < njobs; ++j) {
      const size_t bytes = 1 + rng() % 20000;
      if (off + bytes > src.size()) break;
      jobs.push_back({dst.data() + off, src.data() + off, bytes});
      off += bytes;
    }
    if (b % 997 == 0) usleep(300);  // workers go to sleep in between
    fcx::CopyPool::get().run(jobs, threads, (b & 1) != 0);
    if (std::memcmp(dst.data(), src.data(), off) != 0) {
      std::printf("batch %d: wrong bytes\n", b);
      return 1;
    }
  }
  std::printf("COPY_POOL_OK %d batches\n", batches);
  return 0;
}
