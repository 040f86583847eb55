// mock_rccl.cpp -- TEST-ONLY stand-in for librccl.so, loaded by libfcx through
// FCX_RCCL_LIBRARY (fcx_engine.hip, rccl()).
//
// RCCL refuses two ranks on one device, and the development boxes have one GPU, so libfcx's
// N > 1 boundary exchange (atmos_exchange: the in-place and packed all-reduce, the stream
// joins, the signature agreement) could otherwise first run in the driver's 8-GPU bench.
// This library lets 2..16 processes share GPU 0 and makes every collective a host-memory
// all-reduce through one POSIX shared-memory segment:
//
//   ncclAllReduce: wait for the stream, copy the send buffer to this rank's row of the
//   segment, barrier, check that every rank issued the same call (sequence number, count,
//   data type, operation), reduce the rows in rank order, barrier, copy the result back.
//
// Any mismatch in the call sequence returns ncclInvalidUsage on EVERY rank with a message
// naming the ranks' calls, and a rank that does not arrive within FCX_MOCK_RCCL_TIMEOUT_S
// seconds (default 60) fails the waiting ranks with ncclSystemError instead of hanging them.
// FCX_MOCK_RCCL_LOG=<prefix> writes each rank's call sequence to <prefix>.<rank>, one line
// per call: "seq count dtype op".  Not part of the product: nothing but tests loads it.
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

constexpr int kMaxRanks = 16;
constexpr size_t kCap = size_t(1) << 18;  // doubles per rank and call

struct CallRec {
  uint64_t seq;
  uint64_t count;
  int32_t dtype, op;
};

struct Header {
  std::atomic<uint32_t> bar_count;
  std::atomic<uint32_t> bar_gen;
  std::atomic<uint32_t> failed;
  char why[256];
  CallRec rec[kMaxRanks];
};

thread_local std::string g_msg;

// the HIP runtime the process already uses (libfcx's; torch's in the tests)
struct Hip {
  int (*memcpy)(void *, const void *, size_t, int) = nullptr;
  int (*stream_sync)(void *) = nullptr;
  bool ok = false;
};

const Hip &hip() {
  static Hip h = [] {
    Hip x;
    void *lib = dlopen("libamdhip64.so", RTLD_NOW | RTLD_NOLOAD);
    if (!lib) lib = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) return x;
    x.memcpy = reinterpret_cast<decltype(x.memcpy)>(dlsym(lib, "hipMemcpy"));
    x.stream_sync = reinterpret_cast<decltype(x.stream_sync)>(dlsym(lib, "hipStreamSynchronize"));
    x.ok = x.memcpy && x.stream_sync;
    return x;
  }();
  return h;
}

double timeout_s() {
  const char *t = std::getenv("FCX_MOCK_RCCL_TIMEOUT_S");
  const double v = t ? std::atof(t) : 0.0;
  return v > 0 ? v : 60.0;
}

}  // namespace

struct ncclComm {
  int rank = 0, nranks = 0;
  std::string name;
  size_t bytes = 0;
  Header *h = nullptr;
  double *rows = nullptr;  // [nranks][kCap]
  uint64_t seq = 0;
  FILE *log = nullptr;
};

namespace {

ncclResult_t failed(ncclComm *c, ncclResult_t r, const char *fmt, ...) __attribute__((format(printf, 3, 4)));
ncclResult_t failed(ncclComm *c, ncclResult_t r, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_msg = buf;
  if (c && c->h && c->h->failed.exchange(1) == 0) snprintf(c->h->why, sizeof c->h->why, "rank %d: %s", c->rank, buf);
  return r;
}

// sense-reversing barrier over the segment; false on timeout or when another rank failed
bool barrier(ncclComm *c) {
  Header *h = c->h;
  const uint32_t g = h->bar_gen.load(std::memory_order_acquire);
  if (h->bar_count.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)c->nranks) {
    h->bar_count.store(0, std::memory_order_relaxed);
    h->bar_gen.fetch_add(1, std::memory_order_release);
    return true;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const double limit = timeout_s();
  while (h->bar_gen.load(std::memory_order_acquire) == g) {
    if (h->failed.load(std::memory_order_acquire)) {
      g_msg = std::string("another rank failed: ") + h->why;
      return false;
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
      failed(c, ncclSystemError, "rank %d waited %.0f s at call %llu for the other ranks", c->rank, limit,
             (unsigned long long)c->seq);
      return false;
    }
    usleep(20);
  }
  return true;
}

const char *op_name(int op) { return op == ncclSum ? "sum" : op == ncclMax ? "max" : "other"; }

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
  if (!id) return ncclInvalidArgument;
  unsigned long long r = 0;
  if (FILE *f = std::fopen("/dev/urandom", "rb")) {
    if (std::fread(&r, sizeof r, 1, f) != 1) r = 0;
    std::fclose(f);
  }
  r ^= (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count();
  std::memset(id->internal, 0, sizeof id->internal);
  snprintf(id->internal, sizeof id->internal, "/fcxmock-%d-%llx", (int)getpid(), r);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  if (!hip().ok) return failed(nullptr, ncclSystemError, "mock RCCL: no HIP runtime in the process");
  auto *c = new ncclComm();
  c->rank = rank;
  c->nranks = nranks;
  c->name.assign(id.internal, strnlen(id.internal, sizeof id.internal));
  if (c->name.empty() || c->name[0] != '/') {
    delete c;
    return failed(nullptr, ncclInvalidArgument, "mock RCCL: unique id not from this library");
  }
  c->bytes = sizeof(Header) + 64 + (size_t)nranks * kCap * sizeof(double);
  const int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, (off_t)c->bytes) != 0) {
    if (fd >= 0) close(fd);
    delete c;
    return failed(nullptr, ncclSystemError, "mock RCCL: shared memory %s", id.internal);
  }
  void *p = mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    delete c;
    return failed(nullptr, ncclSystemError, "mock RCCL: mmap");
  }
  c->h = static_cast<Header *>(p);
  c->rows = reinterpret_cast<double *>(static_cast<char *>(p) + (sizeof(Header) + 63) / 64 * 64);
  if (const char *pre = std::getenv("FCX_MOCK_RCCL_LOG")) {
    const std::string path = std::string(pre) + "." + std::to_string(rank);
    c->log = std::fopen(path.c_str(), "w");
  }
  if (!barrier(c)) {  // every rank attached
    munmap(c->h, c->bytes);
    delete c;
    return ncclSystemError;
  }
  *comm = c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  if (!c) return ncclSuccess;
  const bool all = !c->h->failed.load() && barrier(c);  // nobody still reads the segment
  if (c->log) std::fclose(c->log);
  munmap(c->h, c->bytes);
  if (c->rank == 0 || !all) shm_unlink(c->name.c_str());
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t datatype,
                           ncclRedOp_t op, ncclComm_t c, hipStream_t stream) {
  if (!c) return ncclInvalidArgument;
  if (c->h->failed.load()) return failed(c, ncclInvalidUsage, "communicator failed earlier: %s", c->h->why);
  if (datatype != ncclFloat64 || (op != ncclSum && op != ncclMax))
    return failed(c, ncclInvalidArgument, "mock RCCL: only float64 sum / max");
  if (count > kCap) return failed(c, ncclInvalidArgument, "mock RCCL: %zu values > %zu", count, kCap);
  const uint64_t seq = c->seq++;
  if (c->log) {
    std::fprintf(c->log, "%llu %zu %d %s\n", (unsigned long long)seq, count, (int)datatype, op_name(op));
    std::fflush(c->log);
  }
  if (hip().stream_sync(stream) != 0) return failed(c, ncclUnhandledCudaError, "hipStreamSynchronize");
  double *mine = c->rows + (size_t)c->rank * kCap;
  if (count && hip().memcpy(mine, sendbuff, count * sizeof(double), 4 /* hipMemcpyDefault */) != 0)
    return failed(c, ncclUnhandledCudaError, "hipMemcpy of the send buffer");
  c->h->rec[c->rank] = CallRec{seq, (uint64_t)count, (int32_t)datatype, (int32_t)op};
  if (!barrier(c)) return ncclSystemError;
  for (int r = 0; r < c->nranks; ++r) {
    const CallRec &a = c->h->rec[r], &b = c->h->rec[c->rank];
    if (a.seq != b.seq || a.count != b.count || a.dtype != b.dtype || a.op != b.op) {
      // every rank compares every record, so every rank fails this call
      std::string calls;
      for (int q = 0; q < c->nranks; ++q) {
        char one[96];
        snprintf(one, sizeof one, "%srank %d: call %llu, %llu values, %s", q ? "; " : "", q,
                 (unsigned long long)c->h->rec[q].seq, (unsigned long long)c->h->rec[q].count,
                 op_name(c->h->rec[q].op));
        calls += one;
      }
      g_msg = "mock RCCL: ranks issued different collectives (" + calls + ")";
      if (c->h->failed.exchange(1) == 0) snprintf(c->h->why, sizeof c->h->why, "%s", g_msg.c_str());
      return ncclInvalidUsage;
    }
  }
  std::vector<double> res(mine, mine + count);
  for (size_t i = 0; i < count; ++i) {
    double acc = c->rows[i];  // rank order, the same sum on every rank
    for (int r = 1; r < c->nranks; ++r) {
      const double x = c->rows[(size_t)r * kCap + i];
      acc = op == ncclSum ? acc + x : (x > acc ? x : acc);
    }
    res[i] = acc;
  }
  if (!barrier(c)) return ncclSystemError;  // every rank has read every row
  if (count && hip().memcpy(recvbuff, res.data(), count * sizeof(double), 4) != 0)
    return failed(c, ncclUnhandledCudaError, "hipMemcpy of the result");
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

const char *ncclGetErrorString(ncclResult_t r) {
  if (r == ncclSuccess) return "success";
  return g_msg.empty() ? "mock RCCL error" : g_msg.c_str();
}

}  // extern "C"
