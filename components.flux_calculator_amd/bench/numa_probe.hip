// numa_probe.hip -- measurement tool (round 6): does the NUMA node of page-locked host memory
// decide the host-link rate?  Device->host copies into hipHostMalloc memory ran at ~23 GB/s
// for some allocations and ~52 GB/s for others in one process (d2h_flags_probe,
// zc_flags_probe), which flag sets alone did not explain.  Here: the GPU's NUMA node (sysfs
// of its PCI device), the nodes of the CPUs this process may run on, then for the default
// policy (several allocations in a row) and for memory bound to each node (set_mempolicy
// MPOL_BIND + hipHostMallocNumaUser): the node the pages landed on (get_mempolicy), and the
// Baltic step's copies (6.8 MB up, 5.2 MB down, both at once) and the zero-copy kernel step.
//
//   hipcc --offload-arch=gfx950 -O2 numa_probe.hip -o numa_probe && ./numa_probe
#include <hip/hip_runtime.h>

#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

static int read_int(const std::string &path) {
  FILE *f = std::fopen(path.c_str(), "r");
  if (!f) return -2;
  int v = -2;
  if (std::fscanf(f, "%d", &v) != 1) v = -2;
  std::fclose(f);
  return v;
}

static int cpu_node(int cpu) {
  for (int n = 0; n < 16; ++n) {
    const std::string p = "/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/node" + std::to_string(n);
    if (access(p.c_str(), F_OK) == 0) return n;
  }
  return -1;
}

static int page_node(void *p) {  // get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR)
  int node = -1;
  if (syscall(SYS_get_mempolicy, &node, nullptr, 0, p, 3) != 0) return -1;
  return node;
}

__global__ void zc_step(const double2 *in, int nin, double2 *out, int nout, int n2) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n2) return;
  double2 s = make_double2(0.0, 0.0);
  for (int k = 0; k < nin; ++k) {
    const double2 v = in[(size_t)k * n2 + j];
    s.x += v.x;
    s.y += v.y;
  }
  for (int k = 0; k < nout; ++k) out[(size_t)k * n2 + j] = make_double2(s.x + k, s.y + k);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 150;
  const int n = 32768, nin = 26, nout = 20;
  const size_t tin = (size_t)nin * n * 8, tout = (size_t)nout * n * 8, tot = tin + tout;
  char bdf[64] = {0};
  CHECK(hipDeviceGetPCIBusId(bdf, sizeof bdf, 0));
  for (char *c = bdf; *c; ++c) *c = (char)std::tolower(*c);
  const int gpu_node = read_int(std::string("/sys/bus/pci/devices/") + bdf + "/numa_node");
  cpu_set_t set;
  sched_getaffinity(0, sizeof set, &set);
  std::vector<int> nodes_of_cpus(16, 0);
  int ncpu = 0;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &set)) {
      ++ncpu;
      const int nd = cpu_node(c);
      if (nd >= 0 && nd < 16) nodes_of_cpus[nd]++;
    }
  int nnodes = 0;
  while (nnodes < 16 && access(("/sys/devices/system/node/node" + std::to_string(nnodes)).c_str(), F_OK) == 0) ++nnodes;
  std::printf("{\"tool\": \"numa_probe.hip\", \"gpu_pci\": \"%s\", \"gpu_numa_node\": %d, \"numa_nodes\": %d, "
              "\"affinity_cpus\": %d, \"affinity_cpus_per_node\": [",
              bdf, gpu_node, nnodes, ncpu);
  for (int i = 0; i < std::max(nnodes, 1); ++i) std::printf("%s%d", i ? ", " : "", nodes_of_cpus[i]);
  std::printf("], \"runs\": [");
  hipStream_t sa, sb;
  CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  char *d;
  CHECK(hipMalloc((void **)&d, tot));
  CHECK(hipMemset(d, 0, tot));
  struct Run {
    std::string name;
    int bind;  // -1: default policy
    unsigned flags;
  };
  std::vector<Run> runs;
  for (int i = 0; i < 3; ++i) runs.push_back({"default_" + std::to_string(i), -1, hipHostMallocMapped});
  for (int i = 0; i < 2; ++i) runs.push_back({"portable_" + std::to_string(i), -1, hipHostMallocMapped | hipHostMallocPortable});
  for (int nd = 0; nd < nnodes; ++nd) runs.push_back({"bind_node" + std::to_string(nd), nd, hipHostMallocMapped | hipHostMallocNumaUser});
  bool first = true;
  for (const Run &run : runs) {
    if (run.bind >= 0) {
      unsigned long mask = 1ul << run.bind;
      if (syscall(SYS_set_mempolicy, 2 /* MPOL_BIND */, &mask, 64) != 0) continue;
    }
    char *h = nullptr, *hd = nullptr;
    const hipError_t e = hipHostMalloc((void **)&h, tot, run.flags);
    if (run.bind >= 0) syscall(SYS_set_mempolicy, 0 /* MPOL_DEFAULT */, nullptr, 0);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      continue;
    }
    CHECK(hipHostGetDevicePointer((void **)&hd, h, 0));
    std::memset(h, 1, tot);
    const int pn0 = page_node(h), pn1 = page_node(h + tin);
    double res[4];
    for (int c = 0; c < 4; ++c) {
      std::vector<double> t;
      for (int r = 0; r < reps + 10; ++r) {
        const double t0 = now_us();
        if (c == 0 || c == 2) CHECK(hipMemcpyAsync(d, h, tin, hipMemcpyDefault, sa));
        if (c == 1 || c == 2) CHECK(hipMemcpyAsync(h + tin, d + tin, tout, hipMemcpyDefault, sb));
        if (c == 3)
          zc_step<<<(n / 2 + 255) / 256, 256, 0, sa>>>(reinterpret_cast<const double2 *>(hd), nin,
                                                        reinterpret_cast<double2 *>(hd + tin), nout, n / 2);
        CHECK(hipStreamSynchronize(sa));
        CHECK(hipStreamSynchronize(sb));
        if (r >= 10) t.push_back(now_us() - t0);
      }
      std::sort(t.begin(), t.end());
      res[c] = t[t.size() / 2];
    }
    std::printf("%s{\"run\": \"%s\", \"pages_on_node\": [%d, %d], \"dma_up_us\": %.1f, \"dma_down_us\": %.1f, "
                "\"dma_both_us\": %.1f, \"zero_copy_step_us\": %.1f}",
                first ? "" : ", ", run.name.c_str(), pn0, pn1, res[0], res[1], res[2], res[3]);
    first = false;
    CHECK(hipHostFree(h));
  }
  std::printf("]}\n");
  return 0;
}
