// fcx_engine.hip -- host side of libfcx: the C ABI of include/fcx.h.
//
// The engine mirrors the reference data model (local_field(0:10,3)%var(35), basic:86-103):
// every bound slot points at a caller array; identical pointers are aliases and share one
// device buffer (the reference's pointer aliasing, basic:334-358 / prepare:36-38).  At
// fcx_commit the planner validates the bindings against the flux_calculator_prepare.F90
// rules, allocates one device mirror per distinct host array (one pooled hipMalloc, 256-B
// aligned sub-buffers), and builds device parameter blocks for the fused launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include <sched.h>
#include <unistd.h>

#include "fcx_copy_pool.h"
#include "fcx_internal.h"

using namespace fcx;

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(FCX_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

const char *kVarNames[kNumVars] = {
    "ALBE", "ALBA", "AMOI", "AMOM", "FARE", "FICE", "PATM", "PSUR", "QATM", "TATM", "TSUR", "UATM",
    "VATM", "U10M", "V10M", "CMOM", "CMOI", "CHEA", "QSUR", "HLAT", "HSEN", "MEVA", "MPRE", "MRAI",
    "MSNO", "RBBR", "RLWD", "RLWU", "RSID", "RSIU", "RSIN", "RSDD", "RSDR", "UMOM", "VMOM"};

// Where a device mirror sits inside its pool, and so its image in the staging arena
// (FCX_OPT_HOST_STAGING): pool `sp` of the engine's StagePools, byte offset `soff` from the
// pool's base (tiled pools: the slot's offset in the first tile row).  sp < 0: the mirror is
// fed by direct copies (fcx_host_malloc memory, or staging off).
struct StageRef {
  int sp = -1;
  size_t soff = 0;
};

struct Buffer {
  double *host = nullptr;  // caller array (nullptr for device-bound)
  double *dev = nullptr;   // device memory (engine pool or caller's)
  int64_t n = 0;
  bool external = false;   // caller-owned device memory (or a host array used in place)
  bool in_place = false;   // a host array the kernels use through its mapped address
  StageRef st;
  int span = -1;           // fcx_host_malloc array moved by the span transport: its Span
};

// The span transport (FCX_OPT_LIB_SPANS) of fcx_host_malloc arrays: one device buffer per
// host slab the engine's arrays sit in, laid out like the host memory from `lo` on, so that
// arrays adjacent in host memory are adjacent on the device and move as ONE copy.
struct Span {
  uintptr_t lo = 0;  // host address of the device buffer's first byte
  char *dev = nullptr;
  size_t bytes = 0;
};

// A device pool with host-bound mirrors and its page-locked host image: the same bytes at
// the same offsets, so a contiguous run of mirrors is one DMA.  Tiled pools (the field
// mirrors of FCX_OPT_TILED_LAYOUT, the tiled atmosphere outputs) are rows of `pitch` bytes
// (one layout tile of every slot), slot k at k * slot bytes of every row; plain pools hold
// each mirror contiguously.
struct StagePool {
  char *dev = nullptr, *host = nullptr;
  size_t bytes = 0;
  bool tiled = false;
  size_t slot = 0, pitch = 0;  // tiled: bytes of one slot's tile, bytes of one row
  bool mapped = false;         // the image IS the kernels' buffer (device-mapped): no DMA
  bool disabled = false;       // its image could not be page-locked: members take the direct path
};

// One host array <-> its mirror through the staging arena: `n` elements of `es` bytes.
struct Xfer {
  int sp;
  size_t soff;
  char *host;
  int64_t n;
};

struct Csr {
  bool set = false;
  int64_t n_dst = 0;
  std::vector<int32_t> row_ptr, col;
  std::vector<double> w;
  int32_t *d_row = nullptr, *d_col = nullptr;
  double *d_w = nullptr;
};

struct Plan {
  Params host{};
  Params *dev = nullptr;
  std::vector<int> reads, writes;  // buffer ids
  int variant = 0;                 // T=1 specialisation (LaunchConfig::variant)
  bool atm_fused = false;          // exchange -> atmosphere accumulation inside the launch
  AtmosFused af{};
  int atm_nf = 0;
  int atm_phase = 0;               // the phase whose fields the fused accumulation writes
  // remap records written by this launch (host.rec): the launch group `rec_group` of remap
  // `rec_remap` gathers them (plan_fused_records); -1 = none
  int rec_remap = -1, rec_group = -1;
};

int var0(int var) { return var - 1; }

// threads of the host copies: FCX_OPT_HOST_THREADS, else min(16, OMP_NUM_THREADS if set, else
// the CPUs this process may run on) -- an MPI rank pinned to one core copies alone
// an unpinned rank (affinity = every online CPU) shares the node with the other local ranks
// of its launch (MPI or torchrun environment): its share of the CPUs, so that several ranks'
// copy threads do not oversubscribe the cores the coupled models run on
int local_ranks() {
  for (const char *v : {"OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "SLURM_NTASKS_PER_NODE", "LOCAL_WORLD_SIZE"})
    if (const char *x = std::getenv(v)) {
      const int k = std::atoi(x);
      if (k > 0) return k;
    }
  return 1;
}

int default_host_threads() {
  static const int n = [] {
    int cpus = 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = std::max(1, CPU_COUNT(&set));
    const long online = sysconf(_SC_NPROCESSORS_ONLN);
    if (online > 0 && cpus >= online) cpus = std::max(1, cpus / local_ranks());
    if (const char *omp = std::getenv("OMP_NUM_THREADS")) {
      const int t = std::atoi(omp);
      if (t > 0) cpus = std::min(cpus, t);
    }
    return std::max(1, std::min(cpus, 16));
  }();
  return n;
}

}  // namespace

// fcx_upload_field: one host thread per engine that stages the fields the host hands over one
// by one (gather into the arena, DMA on the engine stream) while the host receives the next
struct FieldUploader {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv, idle;
  std::deque<int> q;  // buffer ids
  int busy = 0;
  bool stop = false;
  bool prepared = false;  // this step's arena preconditions are met (stage_in's waits)
  bool dma = false;       // a DMA out of the arena was queued since the last join
  int err = 0;
  std::string msg;
};

struct fcx_engine {
  int device = 0;
  int T = 0;
  int64_t n[3] = {0, 0, 0};
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int8_t method[FCX_NUM_FLUXES][kMaxTypes] = {};
  int slot[kMaxTypes + 1][3][kNumVars];
  bool allocated[kMaxTypes + 1][3][kNumVars] = {};
  uint8_t put_to[kMaxTypes + 1][3][kNumVars] = {};
  std::vector<Buffer> bufs;
  std::map<const double *, int> by_ptr;
  bool committed = false;
  bool any_regrid = false;
  bool aligned16 = true;
  bool f32 = false;       // FCX_PRECISION_F32: float fields, fp32 kernels
  size_t esize = 8;       // bytes per field element
  // bias corrections (bias_corrections.F90)
  bool lcorr = false;
  int32_t init_date = 0;
  std::vector<double> corr_mm;  // [12][n_t]
  void *corr_dev = nullptr;  // [12][n_t] in the engine precision
  Csr rg[4];
  std::vector<std::pair<int, std::pair<int, int>>> averages;  // (phase, (grid, var))
  std::map<std::pair<uint32_t, int>, Plan> plans;               // (stages, avg phase mask)
  void *pool = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  bool gpu_ready = false;
  bool user_stream = false;
  LaunchConfig launch;      // fcx_set_option
  bool specialize = true;
  // exchange -> atmosphere accumulation
  struct AtmosField {
    int phase, s, g, var;
    double *out_host = nullptr, *out_dev = nullptr;
    bool external = false;
    StageRef st;
  };
  int64_t n_atmos = -1;
  std::vector<int32_t> atm_row, atm_col;
  std::vector<double> atm_w;
  bool atm_contiguous = true;
  int32_t *d_atm_row = nullptr, *d_atm_col = nullptr, *d_atm_idx = nullptr;
  // the fused path's maps (which launch reads which: compact_map): a 4-B index per cell
  // (d_atm_idx) and the compacted map (AtmosFused::seg_*: [words] start bits, [words + 1]
  // prefix counts, [segments] atmosphere cells, one allocation)
  void *d_atm_seg = nullptr;
  int32_t *d_atm_tile_a0 = nullptr;  // the compacted map's first cell of every wave tile
  int64_t atm_seg_words = 0, atm_segments = 0;
  std::vector<int32_t> atm_idx;
  // atmosphere cells without exchange cells (land, on a real intersection grid): the fused
  // accumulation has no segment for them, so their zero sums are stored after its launch
  std::vector<int32_t> atm_empty;
  int32_t *d_atm_empty = nullptr;
  int32_t atm_maxseg = 0;
  double *d_atm_xrec = nullptr;    // [tiles][kXRec] crossing records (fix-up kernel)
  int64_t atm_crossings = 0;       // 128-cell tile boundaries inside a segment of the map
  bool atm_halo = true;            // FCX_OPT_ATMOS_HALO: halo tiles where they apply
  double *d_atm_w = nullptr;
  std::vector<AtmosField> atm_fields;
  double *atm_shared = nullptr;
  int32_t atm_nb = 0, atm_stride = 0, atm_left = -1, atm_right = -1;
  bool own_shared = false;        // fcx_set_atmos_boundaries: the engine allocates the slots
  double *atm_shared_own = nullptr;
  struct fcx_comm *comm = nullptr;  // fcx_set_comm: the engine completes its boundary slots
  bool atm_done = false;            // the accumulation of the current run has been launched
  bool exchanged = false;           // ... and its boundary slots completed (comm attached)
  void *atm_pool = nullptr;
  int64_t atm_out_tpad = 0;  // tile-blocked atmosphere outputs (kernels: tiled(a, atm_out_tpad))
  bool atmos_in_run = true;
  bool atm_done_fused = false;  // the last fcx_run already accumulated the atmosphere fields
  int group_members = 0;        // engines in the merged launch of its last run (0: fcx_run)
  std::unique_ptr<FieldUploader> uploader;  // fcx_upload_field
  std::vector<char> field_sent;             // buffers fcx_upload_field staged for the coming run
  // exchange -> model remaps (SCRIP links, CSR by destination in link order)
  struct RemapField {
    int phase, s, g, var;
    double *out_host = nullptr, *out_dev = nullptr;
    bool external = false;
    StageRef st;
  };
  struct Remap {
    int64_t n_dst = 0, n_links = 0;
    int32_t max_src = -1;
    std::vector<int32_t> row, col;
    std::vector<double> w;
    int32_t *d_row = nullptr, *d_col = nullptr;
    double *d_w = nullptr;
    std::vector<RemapField> fields;
    void *pool = nullptr;
    size_t pool_bytes = 0;
    // gather scatter of the map: distinct 64-B segments of a field array (8 fp64 cells) the
    // links of a 256-destination block touch, per link (sampled at commit).  About 0.3 on
    // the geometric and the 1-link synthetic maps, 0.66 on the shuffled 2-link map.
    double scatter = 0.0;
  };
  std::vector<Remap> remaps;
  int remap_pack = 2;        // FCX_OPT_REMAP_PACK: 0 never, 1 always, 2 launches of >= 2 fields
  void *d_rec = nullptr;     // remap records scratch (pack_records), shared by every remap launch
  size_t rec_bytes = 0;
  const Plan *rec_plan = nullptr;  // the whole-phase plan the current run launched (its records)
  bool rec_written = false;        // the last flux launch wrote its plan's remap records
  // host-bound steps: the H2D / compute / D2H pipeline
  int chunks = 8;                                   // fcx_step pipeline depth (1 = off)
  int64_t min_chunk = 256 * 1024;                   // cells per chunk at least (~2 MB/array)
  // kernels use the host arrays in place: 0 off, 1 on, 2 auto (default: grids below two
  // pipeline chunks, where per-array copy calls dominate the step, and only when page-locking
  // is allowed)
  int zero_copy = 2;
  bool zc_active = false;        // some field array is used in place (host-mapped)
  int64_t zc_bytes = 0;          // bytes of host arrays used in place
  // ev0/ev1 around every run (fcx_last_kernel_ms).  Off by default: on the 32K-cell grid the
  // two event records per run made the 3-variant step 41 us instead of 16.5 us
  bool timing = false;
  hipStream_t s_in = nullptr, s_out = nullptr;      // copy streams of the pipeline
  std::vector<hipEvent_t> ev_in, ev_comp, ev_out;   // per chunk
  // staging arena of caller heap arrays (FCX_OPT_HOST_STAGING): page-locked host images of
  // the device pools that hold their mirrors, allocated at the first staged transfer
  bool staging = true;
  bool deferred_scatter = false;        // FCX_OPT_DEFERRED_SCATTER: downloads scattered at fcx_synchronize
#ifdef FCX_AB_BUILD
  bool ab_fixup_each = false;
  bool ab_no_head = false;
#endif
  int host_threads = 0;                 // FCX_OPT_HOST_THREADS (0: default_host_threads)
  std::vector<StagePool> spools;
  std::vector<Xfer> pending_out;        // D2H into the arena whose scatter waits for the stream
  hipEvent_t ev_stage_in = nullptr;     // the last H2D out of the arena
  bool stage_in_live = false;
  size_t pool_bytes = 0, tiled_bytes = 0, atm_pool_bytes = 0;  // device pool sizes
  // tile-blocked mirrors (FCX_OPT_TILED_LAYOUT): tpad = tile stride - kLayoutTile elements,
  // 0 when the field buffers are plain contiguous arrays
  bool tiled_opt = true;
  int64_t tpad = 0;
  std::vector<void *> tiled_pools;  // the pools of a tiled engine (alloc_tiled)
  // fcx_plan_check: plans built on the host only (no device memory; bound buffers without a
  // mirror yet stand in with a non-null tag address), audited, and dropped
  bool plan_dry = false;
  // the span transport of fcx_host_malloc arrays (FCX_OPT_LIB_SPANS, default on)
  bool lib_spans = true;
  std::vector<Span> spans;
  std::vector<char> written;  // per buffer: some plan writes it (never part of an upload run)

  fcx_engine() {
    for (auto &a : slot)
      for (auto &b : a)
        for (auto &c : b) c = -1;
  }
  int buf(int s, int g, int var) const { return slot[s][g - 1][var0(var)]; }
  double *dptr(int s, int g, int var) const {
    int b = buf(s, g, var);
    return b < 0 ? nullptr : bufs[b].dev;
  }
};

static void stage_free(fcx_engine *e);

// ------------------------------------------------------------------ utilities

extern "C" const char *fcx_last_error(void) { return g_err.c_str(); }
extern "C" int fcx_version(void) { return FCX_VERSION; }

// the host's abort routine (flux_calculator.F90:883-887: oasis_abort(comp_id, comp_name, msg)),
// called by the drop-in module before it stops the rank, so the coupled job ends together
static std::atomic<fcx_abort_handler> g_abort{nullptr};

extern "C" int fcx_set_abort_handler(fcx_abort_handler handler) {
  g_abort.store(handler);
  return FCX_OK;
}

extern "C" int fcx_abort(const char *message) {
  fcx_abort_handler h = g_abort.load();
  if (!h) return fail(FCX_E_STATE, "no abort handler registered");
  h(message ? message : "");
  return FCX_OK;  // the handler returned (oasis_abort does not)
}

extern "C" int fcx_method_from_string(const char *s, size_t len) {
  if (!s) return -1;
  size_t e = len;
  while (e > 0 && (s[e - 1] == ' ' || s[e - 1] == '\0')) --e;  // trim()
  std::string m(s, e);
  static const char *names[] = {"none", "zero", "copy", "CCLM", "MOM5", "RCO", "water", "ice", "StBo"};
  for (int i = 0; i < 9; ++i)
    if (m == names[i]) return i;
  return -1;
}

// datetime_helpers.py:4-13 (proleptic Gregorian civil-date arithmetic)
static int64_t days_from_civil(int64_t y, int m, int d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

extern "C" int fcx_current_month(int32_t init_date, int64_t seconds, int32_t *month) {
  if (!month) return fail(FCX_E_ARG, "month is NULL");
  const int64_t y = init_date / 10000;
  const int m = (init_date / 100) % 100, d = init_date % 100;
  if (y < 1 || m < 1 || m > 12 || d < 1 || d > 31)
    return fail(FCX_E_ARG, "init_date %d is not YYYYMMDD", (int)init_date);
  int64_t q = seconds / 86400;
  if (seconds % 86400 != 0 && seconds < 0) q -= 1;
  const int64_t z = days_from_civil(y, m, d) + q + 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  *month = (int32_t)(mp < 10 ? mp + 3 : mp - 9);
  return FCX_OK;
}

// ------------------------------------------------------------------ set-up

extern "C" int fcx_create(int device, int num_surface_types, const int32_t grid_size[3],
                          fcx_engine **out) {
  if (!out || !grid_size) return fail(FCX_E_ARG, "NULL argument");
  *out = nullptr;
  if (num_surface_types < 1 || num_surface_types > kMaxTypes)
    return fail(FCX_E_ARG, "num_surface_types=%d outside 1..%d", num_surface_types, kMaxTypes);
  for (int g = 0; g < 3; ++g)
    if (grid_size[g] < 0) return fail(FCX_E_ARG, "grid_size(%d)=%d < 0", g + 1, grid_size[g]);
  // no HIP call here: the device is touched first in fcx_commit, so that the bindings and
  // their validation can be exercised on a host without a GPU
  auto *e = new fcx_engine();
  e->device = device;
  e->T = num_surface_types;
  for (int g = 0; g < 3; ++g) e->n[g] = grid_size[g];
  *out = e;
  return FCX_OK;
}

static void uploader_stop(fcx_engine *e);
static int uploader_join(fcx_engine *e);

extern "C" int fcx_destroy(fcx_engine *e) {
  if (!e) return FCX_OK;
  uploader_stop(e);
  if (!e->gpu_ready) {
    delete e;
    return FCX_OK;
  }
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (auto &kv : e->plans) {
    (void)hipFree(kv.second.dev);
    (void)hipFree(kv.second.host.rec);
  }
  for (auto &r : e->rg) {
    (void)hipFree(r.d_row);
    (void)hipFree(r.d_col);
    (void)hipFree(r.d_w);
  }
  (void)hipFree(e->corr_dev);
  (void)hipFree(e->d_atm_row);
  (void)hipFree(e->d_atm_seg);
  (void)hipFree(e->d_atm_tile_a0);
  (void)hipFree(e->d_atm_idx);
  (void)hipFree(e->d_atm_empty);
  (void)hipFree(e->d_atm_xrec);
  (void)hipFree(e->d_atm_col);
  (void)hipFree(e->d_atm_w);
  (void)hipFree(e->atm_pool);
  (void)hipFree(e->atm_shared_own);
  for (auto &r : e->remaps) {
    (void)hipFree(r.d_row);
    (void)hipFree(r.d_col);
    (void)hipFree(r.d_w);
    (void)hipFree(r.pool);
  }
  (void)hipFree(e->d_rec);
  (void)hipFree(e->pool);
  for (void *p : e->tiled_pools) (void)hipFree(p);
  for (auto &sp : e->spans) (void)hipFree(sp.dev);
  if (e->ev0) (void)hipEventDestroy(e->ev0);
  if (e->ev1) (void)hipEventDestroy(e->ev1);
  for (hipEvent_t ev : e->ev_in) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->ev_comp) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->ev_out) (void)hipEventDestroy(ev);
  stage_free(e);
  if (e->s_in) (void)hipStreamDestroy(e->s_in);
  if (e->s_out) (void)hipStreamDestroy(e->s_out);
  if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return FCX_OK;
}

extern "C" int fcx_set_stream(fcx_engine *e, void *stream) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed)  // handed-over fields queue their DMAs on the current stream
    if (int r = uploader_join(e)) return r;
  if (e->own_stream && e->stream) {
    (void)hipStreamSynchronize(e->stream);
    (void)hipStreamDestroy(e->stream);
  }
  e->stream = reinterpret_cast<hipStream_t>(stream);
  e->own_stream = false;
  e->user_stream = true;
  return FCX_OK;
}

// first device contact of an engine: device, stream, timing events
static int gpu_init(fcx_engine *e) {
  if (e->gpu_ready) return FCX_OK;
  HIP_TRY(hipSetDevice(e->device));
  if (!e->user_stream) {
    HIP_TRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    e->own_stream = true;
  }
  HIP_TRY(hipEventCreate(&e->ev0));
  HIP_TRY(hipEventCreate(&e->ev1));
  e->gpu_ready = true;
  return FCX_OK;
}

extern "C" int fcx_set_method(fcx_engine *e, int flux, int s, int method) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if (flux < 0 || flux >= FCX_NUM_FLUXES) return fail(FCX_E_ARG, "flux %d unknown", flux);
  if (s < 1 || s > e->T) return fail(FCX_E_ARG, "surface_type %d outside 1..%d", s, e->T);
  if (method < FCX_NONE || method > FCX_STBO) return fail(FCX_E_ARG, "method %d unknown", method);
  e->method[flux][s - 1] = (int8_t)method;
  return FCX_OK;
}

extern "C" int fcx_bind_field(fcx_engine *e, int s, int g, int var, double *ptr, int64_t n,
                              int flags) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if (s < 0 || s > kMaxTypes || g < 1 || g > 3 || var < 1 || var > kNumVars)
    return fail(FCX_E_ARG, "slot (%d,%d,%d) out of range", s, g, var);
  if (!ptr) {
    e->slot[s][g - 1][var0(var)] = -1;
    return FCX_OK;
  }
  if (n < e->n[g - 1])
    return fail(FCX_E_ARG, "%s(%d,%s): array of %lld cells shorter than grid_size %lld",
                kVarNames[var0(var)], s, g == 1 ? "t" : g == 2 ? "u" : "v", (long long)n,
                (long long)e->n[g - 1]);
  const bool on_dev = flags & FCX_MEM_DEVICE;
  auto it = e->by_ptr.find(ptr);
  int b;
  if (it == e->by_ptr.end()) {
    Buffer bf;
    bf.n = n;
    if (on_dev) {
      bf.dev = ptr;
      bf.external = true;
      if (reinterpret_cast<uintptr_t>(ptr) % 16) e->aligned16 = false;
    } else {
      bf.host = ptr;
    }
    b = (int)e->bufs.size();
    e->bufs.push_back(bf);
    e->by_ptr[ptr] = b;
  } else {
    b = it->second;
    if (e->bufs[b].external != on_dev)
      return fail(FCX_E_ARG, "pointer bound both as host and as device memory");
    e->bufs[b].n = std::max(e->bufs[b].n, n);
  }
  e->slot[s][g - 1][var0(var)] = b;
  e->allocated[s][g - 1][var0(var)] = (flags & FCX_ALLOCATED) != 0;
  return FCX_OK;
}

extern "C" int fcx_set_corrections(fcx_engine *e, int enabled, int32_t init_date, const double *corr,
                                   int64_t n, int layout) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  e->lcorr = enabled != 0;
  e->init_date = init_date;
  if (!e->lcorr) return FCX_OK;
  int32_t mth;
  if (fcx_current_month(init_date, 0, &mth) != FCX_OK) return FCX_E_ARG;
  if (!corr || n < e->n[0]) return fail(FCX_E_ARG, "corrections: need %lld cells", (long long)e->n[0]);
  const int64_t nt = e->n[0];
  e->corr_mm.assign((size_t)12 * nt, 0.0);
  // device layout [month][cell]: one coalesced month slice per step (the Fortran
  // corrections(1,12,n) puts the 12 months of a cell together, bias:191)
  for (int m = 0; m < 12; ++m)
    for (int64_t j = 0; j < nt; ++j)
      e->corr_mm[(size_t)m * nt + j] =
          layout == FCX_CORR_CELL_MAJOR ? corr[(size_t)j * 12 + m] : corr[(size_t)m * n + j];
  return FCX_OK;
}

extern "C" int fcx_set_regrid_matrix(fcx_engine *e, int which, int64_t nnz, const int32_t *src,
                                     const int32_t *dst, const double *w) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if (which < 0 || which > 3) return fail(FCX_E_ARG, "regrid matrix %d unknown", which);
  static const int from_g[4] = {2, 3, 1, 1}, to_g[4] = {1, 1, 2, 3};
  const int64_t n_src = e->n[from_g[which] - 1], n_dst = e->n[to_g[which] - 1];
  Csr &c = e->rg[which];
  c.set = true;
  c.n_dst = n_dst;
  c.row_ptr.assign((size_t)n_dst + 1, 0);
  for (int64_t k = 0; k < nnz; ++k) {
    if (src[k] < 1 || src[k] > n_src || dst[k] < 1 || dst[k] > n_dst)
      return fail(FCX_E_ARG, "regrid link %lld (%d -> %d) outside the local grids (io:183-191)",
                  (long long)k + 1, src[k], dst[k]);
    c.row_ptr[(size_t)dst[k]]++;
  }
  for (int64_t d = 0; d < n_dst; ++d) c.row_ptr[(size_t)d + 1] += c.row_ptr[(size_t)d];
  c.col.assign((size_t)nnz, 0);
  c.w.assign((size_t)nnz, 0.0);
  std::vector<int32_t> fill(c.row_ptr.begin(), c.row_ptr.end() - 1);
  for (int64_t k = 0; k < nnz; ++k) {  // stable: link order kept inside each row
    const int32_t at = fill[(size_t)dst[k] - 1]++;
    c.col[(size_t)at] = src[k] - 1;
    c.w[(size_t)at] = w[k];
  }
  return FCX_OK;
}

extern "C" int fcx_set_put_to(fcx_engine *e, int s, int g, int var, int mask) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if (s < 0 || s > kMaxTypes || g < 1 || g > 3 || var < 1 || var > kNumVars || mask < 0 || mask > 7)
    return fail(FCX_E_ARG, "bad put_to arguments");
  e->put_to[s][g - 1][var0(var)] = (uint8_t)mask;
  if (mask) e->any_regrid = true;
  return FCX_OK;
}

extern "C" int fcx_add_average(fcx_engine *e, int phase, int g, int var) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if ((phase != FCX_PHASE_EARLY && phase != FCX_PHASE_NORMAL) || g < 1 || g > 3 || var < 1 ||
      var > kNumVars)
    return fail(FCX_E_ARG, "bad average arguments");
  e->averages.push_back({phase, {g, var}});
  return FCX_OK;
}

// ------------------------------------------------------------------ validation

// flux_calculator_prepare.F90: every method's inputs must be ASSOCIATED and its output
// allocated; 'copy' needs the type-1 array.
static int validate(fcx_engine *e) {
  auto need = [&](int s, int g, int var, const char *what) -> int {
    if (e->buf(s, g, var) < 0)
      return fail(FCX_E_MISSING, "Error calculating %s for surface_type %d on the grid %s_grid: "
                                 "lacking %s", what, s, g == 1 ? "t" : g == 2 ? "u" : "v",
                  kVarNames[var0(var)]);
    return FCX_OK;
  };
#define NEED(s, g, v, w)                      \
  do {                                         \
    if (int r_ = need(s, g, v, w)) return r_;  \
  } while (0)
  for (int s = 1; s <= e->T; ++s) {
    for (int k = 0; k < 3; ++k) {
      const int m = e->method[FCX_SPEC_VAPOR_SURFACE_T + k][s - 1];
      const int g = k + 1;
      if (m == FCX_CCLM) {
        NEED(s, g, FCX_FICE, "QSUR"); NEED(s, g, FCX_PSUR, "QSUR"); NEED(s, g, FCX_TSUR, "QSUR");
        NEED(s, g, FCX_QSUR, "QSUR");
      } else if (m == FCX_COPY) {
        NEED(1, g, FCX_QSUR, "QSUR");
      } else if (m != FCX_NONE) {
        return fail(FCX_E_ARG, "QSUR method %d not known", m);
      }
    }
    int m = e->method[FCX_FLUX_MASS_EVAP][s - 1];
    if (m == FCX_CCLM || m == FCX_MOM5) {
      NEED(s, 1, m == FCX_CCLM ? FCX_AMOI : FCX_CMOI, "MEVA");
      for (int v : {FCX_PSUR, FCX_QATM, FCX_QSUR, FCX_TATM, FCX_UATM, FCX_VATM}) NEED(s, 1, v, "MEVA");
    } else if (m == FCX_RCO) {
      for (int v : {FCX_QATM, FCX_TSUR, FCX_UATM, FCX_VATM}) NEED(s, 1, v, "MEVA");
    } else if (m != FCX_NONE && m != FCX_ZERO && m != FCX_COPY) {
      return fail(FCX_E_ARG, "MEVA method %d not known", m);
    }
    if (m != FCX_NONE) NEED(s, 1, FCX_MEVA, "MEVA");
    if (m == FCX_COPY && e->lcorr) {
      const int m1 = e->method[FCX_FLUX_MASS_EVAP][0];
      if (!(m1 == FCX_ZERO || m1 == FCX_CCLM || m1 == FCX_MOM5 || m1 == FCX_RCO))
        return fail(FCX_E_UNSUPPORTED,
                    "MEVA 'copy' with bias corrections needs surface type 1 to compute MEVA");
      if (e->buf(s, 1, FCX_MEVA) != e->buf(1, 1, FCX_MEVA))
        return fail(FCX_E_ARG, "MEVA 'copy' of type %d must alias the type-1 array", s);
    }
    m = e->method[FCX_FLUX_HEAT_LATENT][s - 1];
    if (m == FCX_WATER || m == FCX_ICE) NEED(s, 1, FCX_MEVA, "HLAT");
    else if (m != FCX_NONE && m != FCX_ZERO && m != FCX_COPY)
      return fail(FCX_E_ARG, "HLAT method %d not known", m);
    if (m != FCX_NONE) NEED(s, 1, FCX_HLAT, "HLAT");
    m = e->method[FCX_FLUX_HEAT_SENSIBLE][s - 1];
    if (m == FCX_CCLM || m == FCX_MOM5) {
      NEED(s, 1, m == FCX_CCLM ? FCX_AMOI : FCX_CHEA, "HSEN");
      for (int v : {FCX_PATM, FCX_PSUR, FCX_QATM, FCX_TATM, FCX_TSUR, FCX_UATM, FCX_VATM})
        NEED(s, 1, v, "HSEN");
    } else if (m == FCX_RCO) {
      for (int v : {FCX_TATM, FCX_TSUR, FCX_UATM, FCX_VATM}) NEED(s, 1, v, "HSEN");
    } else if (m != FCX_NONE && m != FCX_ZERO && m != FCX_COPY) {
      return fail(FCX_E_ARG, "HSEN method %d not known", m);
    }
    if (m != FCX_NONE) NEED(s, 1, FCX_HSEN, "HSEN");
    m = e->method[FCX_FLUX_MOMENTUM][s - 1];
    for (int g = 2; g <= 3; ++g) {
      if (m == FCX_CCLM || m == FCX_MOM5) {
        NEED(s, g, m == FCX_CCLM ? FCX_AMOM : FCX_CMOM, "UMOM/VMOM");
        for (int v : {FCX_PSUR, FCX_QSUR, FCX_TSUR, FCX_UATM, FCX_VATM}) NEED(s, g, v, "UMOM/VMOM");
      } else if (m == FCX_RCO) {
        for (int v : {FCX_UATM, FCX_VATM}) NEED(s, g, v, "UMOM/VMOM");
      } else if (m != FCX_NONE && m != FCX_ZERO && m != FCX_COPY) {
        return fail(FCX_E_ARG, "momentum method %d not known", m);
      }
      if (m != FCX_NONE) NEED(s, g, g == 2 ? FCX_UMOM : FCX_VMOM, "UMOM/VMOM");
    }
    m = e->method[FCX_FLUX_RADIATION_BLACKBODY][s - 1];
    if (m == FCX_STBO) NEED(s, 1, FCX_TSUR, "RBBR");
    else if (m != FCX_NONE && m != FCX_ZERO && m != FCX_COPY)
      return fail(FCX_E_ARG, "RBBR method %d not known", m);
    if (m != FCX_NONE) NEED(s, 1, FCX_RBBR, "RBBR");
  }
#undef NEED
  return FCX_OK;
}

// P7 trigger of flux_calculator.F90:913-914/1003-1004 + calc:376
static bool average_applies(const fcx_engine *e, int g, int var) {
  return e->buf(0, g, var) >= 0 && e->T >= 2 && e->buf(2, g, var) >= 0 &&
         e->allocated[0][g - 1][var0(var)];
}

// ------------------------------------------------------------------ planning

static bool is_compute(int m) { return m == FCX_ZERO || m == FCX_CCLM || m == FCX_MOM5 || m == FCX_RCO; }

// Can u/v work be done from the t-grid loads?  (n equal, same buffers, same QSUR methods)
static bool merge_ok(const fcx_engine *e) {
  if (e->n[0] != e->n[1] || e->n[0] != e->n[2]) return false;
  for (int s = 1; s <= e->T; ++s) {
    if (e->method[FCX_SPEC_VAPOR_SURFACE_U][s - 1] != e->method[FCX_SPEC_VAPOR_SURFACE_T][s - 1] ||
        e->method[FCX_SPEC_VAPOR_SURFACE_V][s - 1] != e->method[FCX_SPEC_VAPOR_SURFACE_T][s - 1])
      return false;
    for (int v : {FCX_TSUR, FCX_FICE, FCX_PSUR, FCX_UATM, FCX_VATM, FCX_QSUR})
      for (int g = 2; g <= 3; ++g)
        if (e->buf(s, g, v) >= 0 && e->buf(s, g, v) != e->buf(s, 1, v)) return false;
    for (int v : {FCX_AMOM, FCX_CMOM})
      if (e->buf(s, 3, v) != e->buf(s, 2, v)) return false;
  }
  return true;
}

// The accumulation rides inside the T=1 specialised launch when every registered field of
// the phase is one of the six fluxes that launch holds in registers (AtmosFused order).
static void plan_fused_atmos(fcx_engine *e, Plan &pl, uint32_t stages, int phase) {
  pl.atm_fused = false;
  // (segments longer than half a tile, several hundred exchange cells per atmosphere cell,
  // go to atmos_kernel: one lane summing a long segment would hold up its whole wave; the
  // fp32 engine uses atmos_kernel too)
  // (fp32 engine: T = 1 only, the register averages of several types are fp64-only)
  // (the maps its launches read: compact_map)
  const bool maps = (!compact_map(e->f32, true) || e->d_atm_seg) && (!compact_map(e->f32, false) || e->d_atm_seg) &&
                    (compact_map(e->f32, true) || e->d_atm_idx) && (compact_map(e->f32, false) || e->d_atm_idx);
  if (!pl.variant || !maps || e->atm_maxseg > kTile / 2 || e->any_regrid || phase <= 0 ||
      phase >= 1000 || !e->specialize || (e->f32 && e->T >= 2))
    return;
  const TypeParams &tp = pl.host.type[0];
  AtmosFused af{};
  int nf = 0;
  const bool multi = e->T >= 2;
  if (multi && !pl.host.ravg_on) return;  // several types: only register averages are fused
  for (size_t fi = 0; fi < e->atm_fields.size(); ++fi) {
    const auto &f = e->atm_fields[fi];
    if (!(f.phase & phase)) continue;
    const int b = e->buf(f.s, f.g, f.var);
    int k = -1;
    if (multi) {  // the type-0 averages OASIS sends, held in registers by the kernel
      for (int slot = 0; slot < kFusedFields; ++slot)
        if (f.s == 0 && pl.host.ravg.out[slot] && b >= 0 && e->bufs[b].dev == pl.host.ravg.out[slot]) k = slot;
      if (k < 0 || af.out[k]) return;
      af.out[k] = f.out_dev;
      af.x[k] = e->bufs[b].dev;
      af.scol[k] = (int32_t)fi;
      ++nf;
      continue;
    }
    if (f.s == 1 && f.var == FCX_MEVA && (stages & S_MEVA) && b == e->buf(1, 1, FCX_MEVA)) k = 0;
    if (f.s == 1 && f.var == FCX_HLAT && (stages & S_HLAT) && b == e->buf(1, 1, FCX_HLAT) &&
        (tp.m_hlat == FCX_WATER || tp.m_hlat == FCX_ICE || tp.m_hlat == FCX_ZERO))
      k = 1;
    if (f.s == 1 && f.var == FCX_HSEN && (stages & S_HSEN) && b == e->buf(1, 1, FCX_HSEN)) k = 2;
    if (f.s == 1 && f.var == FCX_RBBR && (stages & S_RBBR) && b == e->buf(1, 1, FCX_RBBR) &&
        (tp.m_rbbr == FCX_STBO || tp.m_rbbr == FCX_ZERO))
      k = 3;
    if (f.s == 1 && f.var == FCX_UMOM && (stages & S_UMOM) && b == e->buf(1, 2, FCX_UMOM)) k = 4;
    if (f.s == 1 && f.var == FCX_VMOM && (stages & S_VMOM) && b == e->buf(1, 3, FCX_VMOM)) k = 5;
    if (k < 0 || af.out[k]) return;  // not in registers (or twice): separate kernel
    af.out[k] = f.out_dev;
    af.x[k] = e->bufs[b].dev;
    af.scol[k] = (int32_t)fi;
    ++nf;
  }
  if (nf == 0) return;
  if (e->d_atm_seg) {
    af.seg_bits = reinterpret_cast<const uint32_t *>(e->d_atm_seg);
    af.seg_pre = reinterpret_cast<const int32_t *>(af.seg_bits + e->atm_seg_words);
    af.seg_atm = af.seg_pre + e->atm_seg_words + 1;
  }
  af.tile_a0 = e->d_atm_tile_a0;
  af.idx = e->d_atm_idx;
  af.w = e->d_atm_w;
  af.xrec = e->d_atm_xrec;
  af.xrec_on = e->atm_crossings > 0;
#ifdef FCX_AB_BUILD
  if (e->ab_no_head) af.xrec_on = 0;
#endif
  af.n_atmos = e->n_atmos;
  af.shared = e->atm_shared;
  af.stride = e->atm_stride;
  af.left = e->atm_left;
  af.right = e->atm_right;
  af.tpad = e->tpad;
  af.out_tpad = e->atm_out_tpad;
  pl.af = af;
  pl.atm_nf = nf;
  pl.atm_phase = phase;
  pl.atm_fused = true;
}

static bool remap_packs(const fcx_engine *e, const fcx_engine::Remap &rm, int nf);
static int rec_width(const fcx_engine *e, int nf);

// Remap records written by the T=1 specialised launch itself (Params::rec).  A remap launch
// group (the fields run_remaps hands one atmos_kernel launch) that would gather packed
// records (remap_packs), and whose fields are all fluxes of surface type 1 the launch holds
// in registers (the six AtmosFused slots), gets its records from the flux kernel: the
// packing pass and its re-read of the fields disappear.  One group per plan.
static int plan_fused_records(fcx_engine *e, Plan &pl, uint32_t stages, int phase) {
  pl.rec_remap = pl.rec_group = -1;
  Params &P = pl.host;
  for (int k = 0; k < 6; ++k) P.rec_pos[k] = -1;
#ifndef FCX_FUSE_RECORDS  // A/B builds: 0 = remap records only from the packing pass
#define FCX_FUSE_RECORDS 1
#endif
  if (!FCX_FUSE_RECORDS || !pl.variant || e->T != 1 || e->f32 || !e->specialize || e->any_regrid || phase <= 0 || phase >= 1000 ||
      e->remap_pack == 0 || e->launch.cells_per_thread != 2 || !e->aligned16 || !P.merged_uv || P.n_max <= 0)
    return FCX_OK;
  const TypeParams &tp = P.type[0];
  auto slot_of = [&](const fcx_engine::RemapField &f) -> int {
    const int b = e->buf(f.s, f.g, f.var);
    if (f.s != 1 || b < 0) return -1;
    if (f.var == FCX_MEVA && (stages & S_MEVA) && b == e->buf(1, 1, FCX_MEVA) && is_compute(tp.m_meva)) return 0;
    if (f.var == FCX_HLAT && (stages & S_HLAT) && b == e->buf(1, 1, FCX_HLAT) && tp.t.hlat &&
        (tp.m_hlat == FCX_WATER || tp.m_hlat == FCX_ICE || tp.m_hlat == FCX_ZERO))
      return 1;
    if (f.var == FCX_HSEN && (stages & S_HSEN) && b == e->buf(1, 1, FCX_HSEN) && tp.t.hsen && is_compute(tp.m_hsen))
      return 2;
    if (f.var == FCX_RBBR && (stages & S_RBBR) && b == e->buf(1, 1, FCX_RBBR) && tp.t.rbbr &&
        (tp.m_rbbr == FCX_STBO || tp.m_rbbr == FCX_ZERO))
      return 3;
    if (f.var == FCX_UMOM && (stages & S_UMOM) && b == e->buf(1, 2, FCX_UMOM) && tp.uv[0].mom && is_compute(tp.m_mom))
      return 4;
    if (f.var == FCX_VMOM && (stages & S_VMOM) && b == e->buf(1, 3, FCX_VMOM) && tp.uv[1].mom && is_compute(tp.m_mom))
      return 5;
    return -1;
  };
  for (size_t ri = 0; ri < e->remaps.size(); ++ri) {
    const auto &rm = e->remaps[ri];
    std::vector<const fcx_engine::RemapField *> grp;
    int gi = 0;
    auto try_group = [&]() -> bool {
      const int nf = (int)grp.size();
      if (!remap_packs(e, rm, nf) || nf > 6) return false;
      int8_t pos[6] = {-1, -1, -1, -1, -1, -1};
      for (int i = 0; i < nf; ++i) {
        const int k = slot_of(*grp[(size_t)i]);
        if (k < 0 || pos[k] >= 0) return false;
        pos[k] = (int8_t)i;
      }
      const int p = rec_width(e, nf);
      HIP_TRY(hipMalloc(&P.rec, (size_t)P.n_max * p * sizeof(double)));
      P.rec_p = p;
      for (int k = 0; k < 6; ++k) P.rec_pos[k] = pos[k];
      pl.rec_remap = (int)ri;
      pl.rec_group = gi;
      return true;
    };
    for (auto &f : rm.fields) {
      if (!(f.phase & phase)) continue;
      grp.push_back(&f);
      if ((int)grp.size() == kMaxAtmosFields) {
        if (try_group()) return FCX_OK;
        grp.clear();
        ++gi;
      }
    }
    if (!grp.empty() && try_group()) return FCX_OK;
  }
  return FCX_OK;
}

// Register slot (AvgSlot) of the type-0 average of (g, var), or -1 when it has to be done
// by re-reading X_s: every surface type must produce X_s in registers in this launch (a
// computing method and a bound output -- not 'none'/'copy'), and one FARE array per type
// (the t grid's) must serve it.
static int ravg_slot(const fcx_engine *e, const Params &P, uint32_t stages, int g, int var) {
  if (e->T < 2) return -1;
  int slot = -1;
  if (g == 1 && var == FCX_MEVA) slot = A_MEVA;
  if (g == 1 && var == FCX_HLAT) slot = A_HLAT;
  if (g == 1 && var == FCX_HSEN) slot = A_HSEN;
  if (g == 1 && var == FCX_RBBR) slot = A_RBBR;
  if (g == 1 && var == FCX_TSUR) slot = A_TSUR;
  if (P.merged_uv && g == 2 && var == FCX_UMOM) slot = A_UMOM;
  if (P.merged_uv && g == 3 && var == FCX_VMOM) slot = A_VMOM;
  if (slot < 0 || P.ravg.out[slot]) return -1;
  for (int s = 1; s <= e->T; ++s) {
    const TypeParams &tp = P.type[s - 1];
    const int fare = e->buf(s, 1, FCX_FARE);
    if (fare < 0 || e->buf(s, g, FCX_FARE) != fare) return -1;
    bool ok = false;
    switch (slot) {
      case A_MEVA: ok = (stages & S_MEVA) && is_compute(tp.m_meva) && tp.t.meva; break;
      case A_HLAT:
        ok = (stages & S_HLAT) && tp.t.hlat &&
             (tp.m_hlat == FCX_WATER || tp.m_hlat == FCX_ICE || tp.m_hlat == FCX_ZERO);
        break;
      case A_HSEN: ok = (stages & S_HSEN) && is_compute(tp.m_hsen) && tp.t.hsen; break;
      case A_RBBR: ok = (stages & S_RBBR) && tp.t.rbbr && (tp.m_rbbr == FCX_STBO || tp.m_rbbr == FCX_ZERO); break;
      case A_UMOM: ok = (stages & S_UMOM) && is_compute(tp.m_mom) && tp.uv[0].mom; break;
      case A_VMOM: ok = (stages & S_VMOM) && is_compute(tp.m_mom) && tp.uv[1].mom; break;
      case A_TSUR: ok = e->buf(s, 1, FCX_TSUR) >= 0; break;
    }
    if (!ok) return -1;
    // the value averaged is the array's value as stored by this launch: the array of X_s
    const int b = e->buf(s, g, var);
    if (b < 0) return -1;
  }
  return slot;
}

// Plan audit (the 'zero'-momentum fault loaded a wind the planner had left
// unbound).  The kernels guard every load by its own pointer, so an unbound input reads
// nothing; this check, run on every plan before its first launch, names the case where a
// method the plan computes would need an input the planner did not bind -- the predicates of
// process() / uv_grid() in fcx_kernels.hip, restated on the parameter block.
static int plan_audit(const fcx_engine *e, const Params &P) {
  const uint32_t st = P.stages;
  if (P.n_max <= 0) return FCX_OK;  // nothing is launched (a rank with an empty task)
  auto need = [&](const void *ptr, int s, const char *what, const char *name) -> int {
    if (ptr) return FCX_OK;
    return fail(FCX_E_STATE, "plan audit: surface type %d: %s would read the unbound %s (stages 0x%x)", s, what, name,
                (unsigned)st);
  };
#define AUD(ptr, what, name)                                \
  do {                                                      \
    if (int r_ = need((ptr), s + 1, (what), (name))) return r_; \
  } while (0)
  auto cclm_like = [](int m) { return m == FCX_CCLM || m == FCX_MOM5; };
  for (int s = 0; s < P.num_types && P.n[0] > 0; ++s) {
    const TypeParams &tp = P.type[s];
    const TGridPtrs &t = tp.t;
    const bool q_t = (st & S_QSUR_T) && tp.m_qsur[0] == FCX_CCLM;
    if ((st & S_RBBR) && t.rbbr && tp.m_rbbr == FCX_STBO) AUD(t.tsur, "RBBR", "TSUR");
    if (q_t) {
      AUD(t.fice, "QSUR(t)", "FICE");
      AUD(t.psur, "QSUR(t)", "PSUR");
      AUD(t.tsur, "QSUR(t)", "TSUR");
    }
    if (st & S_MEVA) {
      if (cclm_like(tp.m_meva)) {
        AUD(tp.m_meva == FCX_CCLM ? t.amoi : t.cmoi, "MEVA", tp.m_meva == FCX_CCLM ? "AMOI" : "CMOI");
        AUD(t.psur, "MEVA", "PSUR");
        AUD(t.qatm, "MEVA", "QATM");
        AUD(t.tatm, "MEVA", "TATM");
        AUD(t.uatm, "MEVA", "UATM");
        AUD(t.vatm, "MEVA", "VATM");
        if (!q_t) AUD(t.qsur_in, "MEVA", "QSUR");
      } else if (tp.m_meva == FCX_RCO) {
        AUD(t.qatm, "MEVA", "QATM");
        AUD(t.tsur, "MEVA", "TSUR");
        AUD(t.uatm, "MEVA", "UATM");
        AUD(t.vatm, "MEVA", "VATM");
      }
    }
    if ((st & S_HLAT) && t.hlat && (tp.m_hlat == FCX_WATER || tp.m_hlat == FCX_ICE) &&
        !((st & S_MEVA) && is_compute(tp.m_meva)))
      AUD(t.meva_in, "HLAT", "MEVA");
    if ((st & S_HSEN) && t.hsen) {
      if (cclm_like(tp.m_hsen)) {
        AUD(tp.m_hsen == FCX_CCLM ? t.amoi : t.chea, "HSEN", tp.m_hsen == FCX_CCLM ? "AMOI" : "CHEA");
        for (auto pn : {std::make_pair((const void *)t.patm, "PATM"), std::make_pair((const void *)t.psur, "PSUR"),
                        std::make_pair((const void *)t.qatm, "QATM"), std::make_pair((const void *)t.tatm, "TATM"),
                        std::make_pair((const void *)t.tsur, "TSUR"), std::make_pair((const void *)t.uatm, "UATM"),
                        std::make_pair((const void *)t.vatm, "VATM")})
          AUD(pn.first, "HSEN", pn.second);
      } else if (tp.m_hsen == FCX_RCO) {
        AUD(t.tatm, "HSEN", "TATM");
        AUD(t.tsur, "HSEN", "TSUR");
        AUD(t.uatm, "HSEN", "UATM");
        AUD(t.vatm, "HSEN", "VATM");
      }
    }
    if ((st & S_RSDR) && t.rsdr) AUD(P.rsdd0, "RSDR", "RSDD(type 0)");
    if (P.merged_uv) {
      bool q_uv = false;
      for (int k = 0; k < 2; ++k)
        if ((st & (k == 0 ? S_QSUR_U : S_QSUR_V)) && tp.m_qsur[1 + k] == FCX_CCLM && tp.uv[k].qsur) {
          q_uv = true;
          AUD(t.fice, k ? "QSUR(v)" : "QSUR(u)", "FICE");
          AUD(t.psur, k ? "QSUR(v)" : "QSUR(u)", "PSUR");
          AUD(t.tsur, k ? "QSUR(v)" : "QSUR(u)", "TSUR");
        }
      const bool mom = ((st & S_UMOM) && tp.uv[0].mom) || ((st & S_VMOM) && tp.uv[1].mom);
      if (mom && cclm_like(tp.m_mom)) {
        AUD(tp.m_mom == FCX_CCLM ? tp.uv[0].amom : tp.uv[0].cmom, "UMOM/VMOM", tp.m_mom == FCX_CCLM ? "AMOM" : "CMOM");
        AUD(t.psur, "UMOM/VMOM", "PSUR");
        AUD(t.tsur, "UMOM/VMOM", "TSUR");
        AUD(t.uatm, "UMOM/VMOM", "UATM");
        AUD(t.vatm, "UMOM/VMOM", "VATM");
        if (!q_t && !q_uv) AUD(t.qsur_in, "UMOM/VMOM", "QSUR");
      } else if (mom && tp.m_mom == FCX_RCO) {
        AUD(t.uatm, "UMOM/VMOM", "UATM");
        AUD(t.vatm, "UMOM/VMOM", "VATM");
      }
    } else {
      for (int k = 0; k < 2; ++k) {
        if (P.n[1 + k] <= 0) continue;
        const UVGridPtrs &g = tp.uv[k];
        const char *wq = k ? "QSUR(v)" : "QSUR(u)", *wm = k ? "VMOM" : "UMOM";
        const bool do_q = (st & (k == 0 ? S_QSUR_U : S_QSUR_V)) && tp.m_qsur[1 + k] == FCX_CCLM && g.qsur;
        const bool do_m = (st & (k == 0 ? S_UMOM : S_VMOM)) && g.mom;
        if (do_q) {
          AUD(g.fice, wq, "FICE");
          AUD(g.psur, wq, "PSUR");
          AUD(g.tsur, wq, "TSUR");
        }
        if (do_m && cclm_like(tp.m_mom)) {
          AUD(tp.m_mom == FCX_CCLM ? g.amom : g.cmom, wm, tp.m_mom == FCX_CCLM ? "AMOM" : "CMOM");
          AUD(g.psur, wm, "PSUR");
          AUD(g.tsur, wm, "TSUR");
          AUD(g.uatm, wm, "UATM");
          AUD(g.vatm, wm, "VATM");
          if (!do_q) AUD(g.qsur_in, wm, "QSUR");
        } else if (do_m && tp.m_mom == FCX_RCO) {
          AUD(g.uatm, wm, "UATM");
          AUD(g.vatm, wm, "VATM");
        }
      }
    }
    if (P.ravg_on) {
      AUD(P.ravg.fare[s], "type-0 average", "FARE");
      if (P.ravg.out[A_TSUR]) AUD(t.tsur, "type-0 average of TSUR", "TSUR");
    }
    for (int a = 0; a < P.num_avg; ++a) {
      const AvgEntry &ae = P.avg[a];
      AUD(ae.x0, "type-0 average", "type-0 output");
      AUD(ae.x[s], "type-0 average", "averaged field");
      AUD(ae.fare[s], "type-0 average", "FARE");
    }
  }
#undef AUD
  (void)e;
  return FCX_OK;
}

static int build_plan(fcx_engine *e, uint32_t stages, int avg_phases, Plan &pl) {
  Params &P = pl.host;
  std::memset(&P, 0, sizeof P);
  std::set<int> reads, writes;
  for (int g = 0; g < 3; ++g) P.n[g] = e->n[g];
  P.tpad = e->tpad;
  P.num_types = e->T;
  P.stages = stages;
  const bool uv_stages = stages & (S_QSUR_U | S_QSUR_V | S_UMOM | S_VMOM);
  P.merged_uv = uv_stages && merge_ok(e);
  int64_t n_max = 0;
  if (stages & (S_RBBR | S_QSUR_T | S_MEVA | S_HLAT | S_HSEN | S_RSDR)) n_max = e->n[0];
  if (stages & (S_QSUR_U | S_UMOM)) n_max = std::max(n_max, e->n[1]);
  if (stages & (S_QSUR_V | S_VMOM)) n_max = std::max(n_max, e->n[2]);

  // a bound buffer's device address (fcx_plan_check before any mirror exists: a tag address)
  auto dev_of = [&](int b) -> double * {
    if (e->bufs[b].dev || !e->plan_dry) return e->bufs[b].dev;
    return reinterpret_cast<double *>((uintptr_t)(b + 1) << 12);
  };
  // FCX_TEST_PLAN_UNBIND=<VAR> (tests only, fcx_plan_check): the planner "forgets" that input,
  // so the audit's named error can be seen
  const char *unbind = e->plan_dry ? std::getenv("FCX_TEST_PLAN_UNBIND") : nullptr;
  auto in = [&](int s, int g, int var) -> const double * {
    const int b = e->buf(s, g, var);
    if (b < 0) return nullptr;
    if (e->plan_dry && unbind && std::strcmp(unbind, kVarNames[var0(var)]) == 0) return nullptr;
    reads.insert(b);
    return dev_of(b);
  };
  auto out = [&](int s, int g, int var) -> double * {
    const int b = e->buf(s, g, var);
    if (b < 0) return nullptr;
    writes.insert(b);
    return dev_of(b);
  };

  for (int s = 1; s <= e->T; ++s) {
    TypeParams &tp = P.type[s - 1];
    for (int k = 0; k < 3; ++k) tp.m_qsur[k] = e->method[FCX_SPEC_VAPOR_SURFACE_T + k][s - 1];
    tp.m_meva = e->method[FCX_FLUX_MASS_EVAP][s - 1];
    tp.m_hlat = e->method[FCX_FLUX_HEAT_LATENT][s - 1];
    tp.m_hsen = e->method[FCX_FLUX_HEAT_SENSIBLE][s - 1];
    tp.m_mom = e->method[FCX_FLUX_MOMENTUM][s - 1];
    tp.m_rbbr = e->method[FCX_FLUX_RADIATION_BLACKBODY][s - 1];
    TGridPtrs &t = tp.t;
    bool ts = false, fi = false, ps = false, pa = false, qa = false, ta = false, uv = false,
         amoi = false, cmoi = false, chea = false, q_needed = false, me_needed = false;
    const bool q_in_reg = (stages & S_QSUR_T) && tp.m_qsur[0] == FCX_CCLM;
    if (stages & S_RBBR) {
      if (tp.m_rbbr == FCX_STBO) ts = true;
      if (tp.m_rbbr == FCX_STBO || tp.m_rbbr == FCX_ZERO) t.rbbr = out(s, 1, FCX_RBBR);
    }
    if (q_in_reg) {
      fi = ps = ts = true;
      t.qsur = out(s, 1, FCX_QSUR);
    }
    const bool me_in_reg = (stages & S_MEVA) && is_compute(tp.m_meva);
    if (stages & S_MEVA) {
      const int m = tp.m_meva;
      if (m == FCX_CCLM || m == FCX_MOM5) {
        (m == FCX_CCLM ? amoi : cmoi) = true;
        ps = qa = ta = uv = q_needed = true;
      } else if (m == FCX_RCO) {
        qa = ts = uv = true;
      }
      if (is_compute(m)) {
        t.meva = out(s, 1, FCX_MEVA);
        tp.bias_adds = e->lcorr ? 1 : 0;
      }
    }
    if ((stages & S_HLAT) && (tp.m_hlat == FCX_WATER || tp.m_hlat == FCX_ICE || tp.m_hlat == FCX_ZERO)) {
      t.hlat = out(s, 1, FCX_HLAT);
      if (tp.m_hlat != FCX_ZERO) me_needed = true;
    }
    if (stages & S_HSEN) {
      const int m = tp.m_hsen;
      if (m == FCX_CCLM || m == FCX_MOM5) {
        (m == FCX_CCLM ? amoi : chea) = true;
        pa = ps = qa = ta = ts = uv = true;
      } else if (m == FCX_RCO) {
        ta = ts = uv = true;
      }
      if (is_compute(m)) t.hsen = out(s, 1, FCX_HSEN);
    }
    if ((stages & S_RSDR) && e->buf(0, 1, FCX_RSDD) >= 0) {
      bool all = true;
      for (int i = 1; i <= e->T; ++i) all = all && e->buf(i, 1, FCX_RSDR) >= 0;
      if (all) {
        t.rsdr = out(s, 1, FCX_RSDR);
        P.rsdd0 = in(0, 1, FCX_RSDD);
      }
    }
    // u / v grids
    bool mq[2] = {false, false}, mm[2] = {false, false};
    for (int k = 0; k < 2; ++k) {
      const int g = 2 + k;
      UVGridPtrs &gp = tp.uv[k];
      const uint32_t s_q = k == 0 ? S_QSUR_U : S_QSUR_V, s_m = k == 0 ? S_UMOM : S_VMOM;
      mq[k] = (stages & s_q) && tp.m_qsur[1 + k] == FCX_CCLM;
      mm[k] = (stages & s_m) && is_compute(tp.m_mom);
      const bool cclm = tp.m_mom == FCX_CCLM || tp.m_mom == FCX_MOM5;
      if (mq[k]) gp.qsur = out(s, g, FCX_QSUR);
      if (mm[k]) gp.mom = out(s, g, k == 0 ? FCX_UMOM : FCX_VMOM);
      if (P.merged_uv) {
        if (mq[k]) {
          fi = ps = ts = true;
          if (gp.qsur == t.qsur && t.qsur) gp.qsur = nullptr;  // same buffer: stored once
        }
        if (mm[k] && tp.m_mom != FCX_ZERO) {
          uv = true;
          if (cclm) {  // merged: the kernel reads the (shared) coefficient through uv[0]
            ps = ts = q_needed = true;
            if (tp.m_mom == FCX_CCLM) tp.uv[0].amom = in(s, g, FCX_AMOM);
            else tp.uv[0].cmom = in(s, g, FCX_CMOM);
          }
        }
      } else {
        if (mq[k]) {
          gp.fice = in(s, g, FCX_FICE);
          gp.psur = in(s, g, FCX_PSUR);
          gp.tsur = in(s, g, FCX_TSUR);
        }
        if (mm[k] && tp.m_mom != FCX_ZERO) {
          gp.uatm = in(s, g, FCX_UATM);
          gp.vatm = in(s, g, FCX_VATM);
          if (cclm) {
            gp.psur = in(s, g, FCX_PSUR);
            gp.tsur = in(s, g, FCX_TSUR);
            if (tp.m_mom == FCX_CCLM) gp.amom = in(s, g, FCX_AMOM);
            else gp.cmom = in(s, g, FCX_CMOM);
            if (!mq[k]) gp.qsur_in = in(s, g, FCX_QSUR);
          }
        }
      }
    }
    // merged: a momentum stage whose QSUR is not produced in this launch reads QSUR(t)
    const bool q_reg_any = q_in_reg || (P.merged_uv && (mq[0] || mq[1]));
    if (q_needed && !q_reg_any) t.qsur_in = in(s, 1, FCX_QSUR);
    if (q_needed && q_reg_any && !q_in_reg && (stages & S_MEVA) && is_compute(tp.m_meva) &&
        (tp.m_meva == FCX_CCLM || tp.m_meva == FCX_MOM5)) {
      // MEVA runs before QSUR(u/v) in the reference: it must see QSUR(t) as stored
      t.qsur_in = in(s, 1, FCX_QSUR);
    }
    if (me_needed && !me_in_reg) t.meva_in = in(s, 1, FCX_MEVA);
    if (ts) t.tsur = in(s, 1, FCX_TSUR);
    if (fi) t.fice = in(s, 1, FCX_FICE);
    if (ps) t.psur = in(s, 1, FCX_PSUR);
    if (pa) t.patm = in(s, 1, FCX_PATM);
    if (qa) t.qatm = in(s, 1, FCX_QATM);
    if (ta) t.tatm = in(s, 1, FCX_TATM);
    if (uv) {
      t.uatm = in(s, 1, FCX_UATM);
      t.vatm = in(s, 1, FCX_VATM);
    }
    if (amoi) t.amoi = in(s, 1, FCX_AMOI);
    if (cmoi) t.cmoi = in(s, 1, FCX_CMOI);
    if (chea) t.chea = in(s, 1, FCX_CHEA);
  }
  // bias: a 'copy' type adds corr once more to the aliased type-1 array (calc:112-116),
  // which in flux-major order happens before any HLAT reads it
  if (stages & S_MEVA && e->lcorr)
    for (int s = 2; s <= e->T; ++s)
      if (e->method[FCX_FLUX_MASS_EVAP][s - 1] == FCX_COPY) P.type[0].bias_adds++;

  // standard variant of every surface type: the method sets compiled into cells_kernel<.., VAR>
  // (HLAT and RBBR methods stay per type at run time)
  pl.variant = 0;
  if (P.merged_uv) {
    for (int v = 1; v <= 3; ++v) {
      const int m = v == 1 ? FCX_CCLM : v == 2 ? FCX_MOM5 : FCX_RCO;
      const int q = v == 3 ? FCX_NONE : FCX_CCLM;
      bool all = true;
      for (int s = 0; s < e->T; ++s) {
        const TypeParams &tp = P.type[s];
        all = all && tp.m_meva == m && tp.m_hsen == m && tp.m_mom == m && tp.m_qsur[0] == q &&
              tp.m_qsur[1] == q && tp.m_qsur[2] == q;
      }
      if (all) pl.variant = v;
    }
  }

  // type-0 averages
  if (stages & S_AVG) {
    std::vector<std::pair<int, int>> list;
    if (avg_phases >= 1000) {  // explicit average_across_surface_types(g, var) call
      const int g = (avg_phases - 1000) / 100, var = (avg_phases - 1000) % 100;
      if (e->allocated[0][g - 1][var0(var)]) list.push_back({g, var});  // calc:376
    } else {
      for (auto &a : e->averages)
        if ((a.first & avg_phases) && average_applies(e, a.second.first, a.second.second))
          list.push_back(a.second);
    }
    for (auto &a : list) {
      const int g = a.first, var = a.second;
      const int slot = ravg_slot(e, P, stages, g, var);
      if (slot >= 0) {  // accumulated in registers as the types are produced
        P.ravg.out[slot] = out(0, g, var);
        for (int s = 1; s <= e->T; ++s) {
          P.ravg.fare[s - 1] = in(s, 1, FCX_FARE);
          if (slot == A_TSUR) P.type[s - 1].t.tsur = in(s, 1, FCX_TSUR);
        }
        P.ravg_on = 1;
        n_max = std::max(n_max, e->n[0]);
        continue;
      }
      if (P.num_avg >= kMaxAvg) return fail(FCX_E_UNSUPPORTED, "more than %d averaged outputs", kMaxAvg);
      AvgEntry &ae = P.avg[P.num_avg++];
      ae.grid = g - 1;
      ae.x0 = out(0, g, var);
      for (int s = 1; s <= e->T; ++s) {
        if (e->buf(s, g, var) < 0 || e->buf(s, g, FCX_FARE) < 0)
          return fail(FCX_E_MISSING, "average of %s: surface type %d lacks %s or FARE",
                      kVarNames[var0(var)], s, kVarNames[var0(var)]);
        // values produced in this launch are re-read by the same thread (in order)
        ae.x[s - 1] = dev_of(e->buf(s, g, var));
        if (!writes.count(e->buf(s, g, var))) reads.insert(e->buf(s, g, var));
        ae.fare[s - 1] = in(s, g, FCX_FARE);
      }
      n_max = std::max(n_max, e->n[g - 1]);
    }
  }
  P.n_max = n_max;
  pl.reads.assign(reads.begin(), reads.end());
  pl.writes.assign(writes.begin(), writes.end());
  // buffers that are both read and written in the launch are produced there: not inputs
  std::vector<int> pure;
  for (int b : pl.reads)
    if (!writes.count(b)) pure.push_back(b);
  pl.reads.swap(pure);
  if (int r = plan_audit(e, P)) return r;
  if (e->plan_dry) return FCX_OK;  // fcx_plan_check: host only
  plan_fused_atmos(e, pl, stages, avg_phases);
  if (int r = plan_fused_records(e, pl, stages, avg_phases)) return r;
  HIP_TRY(hipMalloc(&pl.dev, sizeof(Params)));
  HIP_TRY(hipMemcpy(pl.dev, &P, sizeof(Params), hipMemcpyHostToDevice));
  return FCX_OK;
}

static uint32_t phase_stages(int phase);
static int staged_sequence(int phase, std::vector<std::pair<uint32_t, int>> &seq);

// Every plan the engine can launch, built on the host and audited (plan_audit), before
// fcx_commit and without a GPU: the whole phases with their averages, the reference
// sequence of a regridding engine, each per-call subroutine and each explicit average.
extern "C" int fcx_plan_check(fcx_engine *e) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "fcx_plan_check runs before fcx_commit");
  if (int r = validate(e)) return r;
  std::vector<std::pair<uint32_t, int>> sets;
  for (int ph : {(int)FCX_PHASE_EARLY, (int)FCX_PHASE_NORMAL, (int)(FCX_PHASE_EARLY | FCX_PHASE_NORMAL)}) {
    sets.push_back({phase_stages(ph), ph});
    std::vector<std::pair<uint32_t, int>> seq;
    staged_sequence(ph, seq);
    for (auto &x : seq) sets.push_back({x.first, 0});
    sets.push_back({S_AVG, ph});
  }
  for (uint32_t st : {S_QSUR_T, S_QSUR_U, S_QSUR_V, S_MEVA, S_HLAT, S_HSEN, S_UMOM, S_VMOM, S_RBBR, S_RSDR})
    sets.push_back({st, 0});
  for (auto &a : e->averages) sets.push_back({S_AVG, 1000 + 100 * a.second.first + a.second.second});
  e->plan_dry = true;
  int rc = FCX_OK;
  for (auto &x : sets) {
    Plan p;
    if ((rc = build_plan(e, x.first, x.second, p)) != FCX_OK) break;
  }
  e->plan_dry = false;
  return rc;
}

static int get_plan(fcx_engine *e, uint32_t stages, int avg_phases, Plan **pl) {
  auto key = std::make_pair(stages, avg_phases);
  auto it = e->plans.find(key);
  if (it == e->plans.end()) {
    Plan p;
    if (int r = build_plan(e, stages, avg_phases, p)) return r;
    it = e->plans.emplace(key, p).first;
  }
  *pl = &it->second;
  return FCX_OK;
}

// Library-owned page-locked host memory (fcx_host_malloc).  A host that allocates its
// local_field arrays here hands the engine memory the library itself locked and mapped at
// allocation, page-exclusive by construction and alive until fcx_host_free: the kernels can
// use it in place (zero-copy) and the copies DMA from it directly, with no registration of
// caller memory at all.
//
// Round 6: the blocks are carved from large page-locked slabs, 256-B aligned, one after the
// other in call order.  A host that allocates its fields the way the reference does --
// every input array first (flux_calculator.F90:436-560, allocate_localvar, basic:288-309),
// then the outputs (do_prepare_calculation, prepare:36-42) -- thereby lays out each phase's
// inputs as one span and its outputs as another, and an engine moves each span with ONE
// copy per direction (the span transport, FCX_OPT_LIB_SPANS) instead of one per array.
namespace {

constexpr size_t kSlabBytes = size_t(32) << 20;  // smallest slab (one Baltic-size engine: ~9 MB)
// Page-locked host memory of the library (slabs, staging images) is allocated PORTABLE.  On
// the shared MI355X boxes a device->host copy of the Baltic step's 5.2 MB ran at ~23 GB/s in
// some allocations and at ~52 GB/s in others, with the host->device rate moving too (128 to
// 172 us for 6.8 MB) from one allocation to the next in one process; neither the allocation
// flags nor the NUMA node of the pages (bound to either node of the box) explained it -- the
// link is shared with the machine's other GPUs' jobs (bench/d2h_flags_probe.hip,
// zc_flags_probe.hip, numa_probe.hip, profiles/r06/probes/).  Portable memory never measured
// slower and is what a multi-device host needs.
#ifndef FCX_PIN_PORTABLE  // A/B builds: 0 = the pre-round-6 flags (hipHostMallocDefault / Mapped)
#define FCX_PIN_PORTABLE 1
#endif
#ifndef FCX_PIN_NONCOHERENT  // A/B builds: 1 = mapped non-coherently (the GPU's L2 may hold host lines
#define FCX_PIN_NONCOHERENT 0  // within a kernel; made visible at the kernel boundaries)
#endif
constexpr unsigned kHostPinFlags = (FCX_PIN_PORTABLE ? hipHostMallocPortable : hipHostMallocDefault) |
                                   (FCX_PIN_NONCOHERENT ? hipHostMallocNonCoherent : 0u);
constexpr size_t kBlockAlign = 256;

struct HostSlab {
  char *host = nullptr, *dev = nullptr;  // page-locked, mapped for the device at allocation
  size_t bytes = 0, used = 0;            // blocks go at `used`, in call order
  int live = 0;
};
struct HostBlock {
  size_t bytes;  // as requested
  uintptr_t slab;
};
std::mutex g_blk_mu;
std::map<uintptr_t, HostSlab> g_slabs;    // keyed by the slab's host address
std::map<uintptr_t, HostBlock> g_blocks;  // keyed by the block's host address
uintptr_t g_cur_slab = 0;                 // the slab new blocks go to (0: none)

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// the block holding [h, h + bytes), under g_blk_mu; end() if none
std::map<uintptr_t, HostBlock>::const_iterator block_of(uintptr_t a, size_t bytes) {
  auto it = g_blocks.upper_bound(a);
  if (it == g_blocks.begin()) return g_blocks.end();
  --it;
  if (a + bytes > it->first + it->second.bytes) return g_blocks.end();
  return it;
}

// device-visible address of [h, h + bytes) if it lies inside one fcx_host_malloc block
void *lib_block_device_ptr(const void *h, size_t bytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(h);
  std::lock_guard<std::mutex> lk(g_blk_mu);
  auto it = block_of(a, bytes);
  if (it == g_blocks.end()) return nullptr;
  const HostSlab &sl = g_slabs.at(it->second.slab);
  return sl.dev + (a - reinterpret_cast<uintptr_t>(sl.host));
}

// the fcx_host_malloc block and slab holding [h, h + bytes): false if none
struct LibBlock {
  uintptr_t start = 0, end = 0, slab = 0;  // block [start, end) as requested, its slab
};
bool lib_block_of(const void *h, size_t bytes, LibBlock *out) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(h);
  std::lock_guard<std::mutex> lk(g_blk_mu);
  auto it = block_of(a, bytes);
  if (it == g_blocks.end()) return false;
  *out = LibBlock{it->first, it->first + it->second.bytes, it->second.slab};
  return true;
}

}  // namespace

extern "C" int fcx_host_malloc(size_t bytes, void **ptr) {
  if (!ptr) return fail(FCX_E_ARG, "ptr is NULL");
  *ptr = nullptr;
  const size_t want = bytes ? bytes : 1, need = round_up(want, kBlockAlign);
  std::lock_guard<std::mutex> lk(g_blk_mu);
  HostSlab *sl = g_cur_slab ? &g_slabs.at(g_cur_slab) : nullptr;
  if (!sl || sl->used + need > sl->bytes) {  // a new slab, the current one from now on
    HostSlab ns;
    ns.bytes = std::max(kSlabBytes, round_up(need, size_t(2) << 20));
    void *h = nullptr, *d = nullptr;
    hipError_t err = hipHostMalloc(&h, ns.bytes, hipHostMallocMapped | kHostPinFlags);
    if (err != hipSuccess) return fail(FCX_E_NOMEM, "hipHostMalloc(%zu): %s", ns.bytes, hipGetErrorString(err));
    err = hipHostGetDevicePointer(&d, h, 0);
    if (err != hipSuccess || !d) {
      (void)hipHostFree(h);
      return fail(FCX_E_HIP, "hipHostGetDevicePointer: %s", hipGetErrorString(err));
    }
    ns.host = static_cast<char *>(h);
    ns.dev = static_cast<char *>(d);
    g_cur_slab = reinterpret_cast<uintptr_t>(h);
    sl = &(g_slabs[g_cur_slab] = ns);
  }
  char *p = sl->host + sl->used;
  sl->used += need;
  ++sl->live;
  g_blocks[reinterpret_cast<uintptr_t>(p)] = HostBlock{want, reinterpret_cast<uintptr_t>(sl->host)};
  *ptr = p;
  return FCX_OK;
}

extern "C" int fcx_host_free(void *ptr) {
  if (!ptr) return FCX_OK;
  void *slab_host = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_blk_mu);
    auto it = g_blocks.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == g_blocks.end()) return fail(FCX_E_ARG, "%p was not allocated by fcx_host_malloc", ptr);
    HostSlab &sl = g_slabs.at(it->second.slab);
    const uintptr_t a = it->first, end = a + round_up(it->second.bytes, kBlockAlign);
    if (end == reinterpret_cast<uintptr_t>(sl.host) + sl.used) sl.used = a - reinterpret_cast<uintptr_t>(sl.host);
    const uintptr_t key = it->second.slab;
    g_blocks.erase(it);
    if (--sl.live == 0) {  // the slab's last block: the slab goes back
      slab_host = sl.host;
      g_slabs.erase(key);
      if (g_cur_slab == key) g_cur_slab = 0;
    }
  }
  if (slab_host) HIP_TRY(hipHostFree(slab_host));
  return FCX_OK;
}

// Zero-copy (FCX_OPT_ZERO_COPY): a host array inside an fcx_host_malloc block is used by the
// kernels in place through its device-visible address -- no device mirror, no copy call; the
// cells kernel streams it over the host link.  For the latency-bound small grids this
// replaces ~17 copy calls per step by one launch.  Caller heap arrays are never used in
// place: GPU access to them goes through a hipHostRegister (userptr) mapping, and twice a
// kernel access through such a mapping missed the page it addressed.
// Every other array keeps a mirror.  Returns the number of arrays used in place.
static int map_host_arrays(fcx_engine *e) {
  auto mapped = [&](void *host, size_t bytes) -> void * { return lib_block_device_ptr(host, bytes); };
  int count = 0;
  for (auto &bf : e->bufs) {
    if (bf.external || !bf.host) continue;
    if (void *d = mapped(bf.host, (size_t)bf.n * e->esize)) {
      bf.dev = reinterpret_cast<double *>(d);
      bf.external = true;  // the engine neither owns nor copies it
      bf.in_place = true;
      e->zc_bytes += bf.n * (int64_t)e->esize;
      ++count;
      if (reinterpret_cast<uintptr_t>(d) % 16) e->aligned16 = false;
    }
  }
  for (auto &f : e->atm_fields) {
    if (f.external || !f.out_host) continue;
    if (void *d = mapped(f.out_host, (size_t)std::max<int64_t>(e->n_atmos, 1) * e->esize)) {
      f.out_dev = reinterpret_cast<double *>(d);
      f.external = true;
      e->zc_bytes += std::max<int64_t>(e->n_atmos, 0) * (int64_t)e->esize;
      ++count;
    }
  }
  for (auto &rm : e->remaps)
    for (auto &f : rm.fields) {
      if (f.external || !f.out_host) continue;
      if (void *d = mapped(f.out_host, (size_t)std::max<int64_t>(rm.n_dst, 1) * e->esize)) {
        f.out_dev = reinterpret_cast<double *>(d);
        f.external = true;
        e->zc_bytes += rm.n_dst * (int64_t)e->esize;
        ++count;
      }
    }
  return count;
}

// The span transport: every fcx_host_malloc array not used in place gets its mirror in the
// device buffer of its slab's span (Span), at its host offset.  Returns the arrays mapped.
static int map_lib_spans(fcx_engine *e, int *count) {
  *count = 0;
  const size_t es = e->esize;
  std::map<uintptr_t, std::vector<int>> by_slab;
  for (size_t b = 0; b < e->bufs.size(); ++b) {
    const Buffer &bf = e->bufs[b];
    if (bf.external || !bf.host || bf.n <= 0) continue;
    LibBlock lb;
    if (lib_block_of(bf.host, (size_t)bf.n * es, &lb)) by_slab[lb.slab].push_back((int)b);
  }
  for (auto &kv : by_slab) {
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    for (int b : kv.second) {
      const uintptr_t h = reinterpret_cast<uintptr_t>(e->bufs[(size_t)b].host);
      lo = std::min(lo, h);
      hi = std::max(hi, h + (size_t)e->bufs[(size_t)b].n * es);
    }
    lo &= ~uintptr_t(kBlockAlign - 1);  // (device offsets keep the host's alignment mod 256)
    Span sp;
    sp.lo = lo;
    sp.bytes = hi - lo;
    hipError_t err = hipMalloc((void **)&sp.dev, sp.bytes);
    if (err != hipSuccess)
      return fail(FCX_E_NOMEM, "hipMalloc(%zu) for a span of fcx_host_malloc arrays: %s", sp.bytes,
                  hipGetErrorString(err));
    const int id = (int)e->spans.size();
    e->spans.push_back(sp);
    for (int b : kv.second) {
      Buffer &bf = e->bufs[(size_t)b];
      bf.dev = reinterpret_cast<double *>(sp.dev + (reinterpret_cast<uintptr_t>(bf.host) - lo));
      bf.external = true;  // not in the engine's pools (the tiled layout is off for it)
      bf.span = id;
      if (reinterpret_cast<uintptr_t>(bf.dev) % 16) e->aligned16 = false;
      ++*count;
    }
  }
  return FCX_OK;
}

// per buffer: written by some plan (a flux output, a type-0 average, a regrid destination)
static void classify_written(fcx_engine *e) {
  static const int kOut[] = {FCX_QSUR, FCX_MEVA, FCX_HLAT, FCX_HSEN, FCX_RBBR, FCX_UMOM, FCX_VMOM, FCX_RSDR};
  e->written.assign(e->bufs.size(), 0);
  for (int s = 0; s <= e->T; ++s)
    for (int g = 1; g <= 3; ++g) {
      for (int v : kOut)
        if (e->buf(s, g, v) >= 0) e->written[(size_t)e->buf(s, g, v)] = 1;
      for (int v = 1; v <= kNumVars; ++v)
        for (int k = 0; k < 3; ++k)
          if (((e->put_to[s][g - 1][v - 1] >> k) & 1) && e->buf(s, k + 1, v) >= 0)
            e->written[(size_t)e->buf(s, k + 1, v)] = 1;
    }
  for (auto &a : e->averages)
    if (e->buf(0, a.second.first, a.second.second) >= 0) e->written[(size_t)e->buf(0, a.second.first, a.second.second)] = 1;
}

// May a copy run continue from host address r1 (one array's end) over the gap to b0 (the next
// array's start)?  Downloads write the host bytes: only over the 256-B padding between two
// consecutive fcx_host_malloc blocks, where no block can ever lie.  Uploads write device bytes
// only: over any gap up to kUploadGap that holds none of the engine's written arrays (whose
// mirrors may hold results not yet downloaded); the rest of the gap -- other inputs, free
// slab, other engines' arrays -- lands in span bytes no mirror of this engine uses or in
// mirrors of inputs, with the host's own values.
constexpr size_t kUploadGap = size_t(512) << 10;  // ~9.9 us at ~53 GB/s: about what one more copy costs (9.4 us)
static bool span_gap_ok(const fcx_engine *e, int span, uintptr_t r1, uintptr_t b0, bool h2d) {
  if (b0 <= r1) return true;
  if (h2d) {
    if (b0 - r1 > kUploadGap) return false;
    for (size_t b = 0; b < e->bufs.size(); ++b) {
      const Buffer &bf = e->bufs[b];
      if (bf.span != span || !e->written[b]) continue;
      const uintptr_t h = reinterpret_cast<uintptr_t>(bf.host), z = h + (size_t)bf.n * e->esize;
      if (h < b0 && z > r1) return false;
    }
    return true;
  }
  if (b0 - r1 >= kBlockAlign) return false;
  LibBlock a, b;
  if (!lib_block_of(reinterpret_cast<const void *>(r1 - 1), 1, &a) || !lib_block_of(reinterpret_cast<const void *>(b0), 1, &b))
    return false;
  return a.end == r1 && b.start == b0 && a.slab == b.slab && round_up(a.end, kBlockAlign) == b0;
}

// the span copies of buffers `ids` (span arrays only): sorted by host address, every run of
// arrays the gap rule joins as ONE hipMemcpyAsync.  runs: the number of copies (queued only
// when s is not null)
static int span_copy(fcx_engine *e, std::vector<int> ids, bool h2d, hipStream_t s, int *runs = nullptr) {
  const size_t es = e->esize;
  std::sort(ids.begin(), ids.end(), [&](int x, int y) { return e->bufs[(size_t)x].host < e->bufs[(size_t)y].host; });
  int nr = 0;
  for (size_t i = 0; i < ids.size();) {
    const Buffer &a = e->bufs[(size_t)ids[i]];
    const int sp = a.span;
    const uintptr_t r0 = reinterpret_cast<uintptr_t>(a.host);
    uintptr_t r1 = r0 + (size_t)a.n * es;
    size_t j = i + 1;
    for (; j < ids.size(); ++j) {
      const Buffer &b = e->bufs[(size_t)ids[j]];
      const uintptr_t b0 = reinterpret_cast<uintptr_t>(b.host);
      if (b.span != sp || !span_gap_ok(e, sp, r1, b0, h2d)) break;
      r1 = std::max(r1, b0 + (size_t)b.n * es);
    }
    ++nr;
    if (s) {
      const Span &p = e->spans[(size_t)sp];
      char *d = p.dev + (r0 - p.lo);
      char *h = reinterpret_cast<char *>(r0);
      HIP_TRY(h2d ? hipMemcpyAsync(d, h, r1 - r0, hipMemcpyDefault, s) : hipMemcpyAsync(h, d, r1 - r0, hipMemcpyDefault, s));
    }
    i = j;
  }
  if (runs) *runs = nr;
  return FCX_OK;
}

// Tile-blocked mirrors (FCX_OPT_TILED_LAYOUT).  Every field array is cut into tiles of
// kLayoutTile cells; tile t of all arrays of one pool sits together: array k of the pool at
// element t * S * kLayoutTile + k * kLayoutTile, S = slots per tile, the same S for every
// pool so that one tile stride serves every field pointer.  Pools by use in the whole-step
// launch (its plan, built here on the bindings): the arrays it only reads, the arrays it
// writes, and the rest (bound but not touched by it, e.g. another variant's coefficients)
// in pools of their own, so a launch touches every slot of the read pool and no gaps sit
// between the arrays it streams.  A wave's accesses then fall in one contiguous region per
// pool instead of 10-20 separate streams: 6.35 vs 5.8 TB/s for the CCLM/MOM5/RCO access
// shapes (bench/layout_probe.hip; one mixed pool 6.28, a pool with unused slots between the
// streamed arrays 6.1, tiles of 2048 / 8192 cells 6.25 / 6.31).
#ifndef FCX_TILED_ATM  // A/B builds: 0 keeps the atmosphere output mirrors contiguous
#define FCX_TILED_ATM 1
#endif
static uint32_t phase_stages(int phase);
static int alloc_tiled(fcx_engine *e) {
  static const int kOut[] = {FCX_QSUR, FCX_MEVA, FCX_HLAT, FCX_HSEN, FCX_RBBR, FCX_UMOM, FCX_VMOM, FCX_RSDR};
  enum { kRead = 0, kWrite = 1, kCold = 2 };
  std::vector<int> cls(e->bufs.size(), kCold);
  {  // the whole-step plan's read and write sets: built on the host only (plan_dry: the
     // mirrors do not exist yet, tag addresses stand in for them), then dropped
    Plan p;
    const std::string saved = g_err;
    e->plan_dry = true;
    if (build_plan(e, phase_stages(FCX_PHASE_EARLY | FCX_PHASE_NORMAL), FCX_PHASE_EARLY | FCX_PHASE_NORMAL, p) ==
        FCX_OK) {
      for (int b : p.reads) cls[b] = kRead;
      for (int b : p.writes) cls[b] = kWrite;
    }
    e->plan_dry = false;
    g_err = saved;
  }
  for (int s = 0; s <= e->T; ++s)  // outputs of other phases / staged launches
    for (int g = 1; g <= 3; ++g)
      for (int v : kOut)
        if (e->buf(s, g, v) >= 0 && cls[e->buf(s, g, v)] == kCold) cls[e->buf(s, g, v)] = kWrite;
  for (auto &a : e->averages) {
    const int b = e->buf(0, a.second.first, a.second.second);
    if (b >= 0 && cls[b] == kCold) cls[b] = kWrite;
  }
  int64_t n_max = 0;
  int count[3] = {0, 0, 0};
  for (size_t b = 0; b < e->bufs.size(); ++b) {
    n_max = std::max(n_max, e->bufs[b].n);
    ++count[cls[b]];
  }
  const int64_t S = std::max(1, std::max(count[kRead], count[kWrite]));
  const int64_t tiles = std::max<int64_t>(1, (n_max + kLayoutTile - 1) / kLayoutTile);
  const size_t bytes = (size_t)tiles * S * kLayoutTile * e->esize;
  e->tiled_bytes = bytes;
  // pool and slot of every buffer: read pool, write pool, then the cold ones S to a pool
  std::vector<std::pair<int, int>> at(e->bufs.size());
  int npools = 0, fill[3] = {0, 0, 0}, pool_of[2] = {-1, -1}, cold_pool = -1;
  for (size_t b = 0; b < e->bufs.size(); ++b) {
    const int c = cls[b];
    if (c != kCold) {
      if (pool_of[c] < 0) pool_of[c] = npools++;
      at[b] = {pool_of[c], fill[c]++};
    } else {
      if (cold_pool < 0 || fill[kCold] == S) cold_pool = npools++, fill[kCold] = 0;
      at[b] = {cold_pool, fill[kCold]++};
    }
  }
  for (int k = 0; k < npools; ++k) {
    void *p = nullptr;
    hipError_t err = hipMalloc(&p, bytes);
    if (err != hipSuccess)
      return fail(FCX_E_NOMEM, "hipMalloc(%zu) for the tiled field mirrors: %s", bytes, hipGetErrorString(err));
    e->tiled_pools.push_back(p);
  }
  for (size_t b = 0; b < e->bufs.size(); ++b)
    e->bufs[b].dev = reinterpret_cast<double *>((char *)e->tiled_pools[at[b].first] +
                                                (size_t)at[b].second * kLayoutTile * e->esize);
  e->tpad = (S - 1) * kLayoutTile;
  return FCX_OK;
}

// Host <-> device copies name no direction (hipMemcpyDefault): the runtime then looks the
// host pointer up and moves page-locked memory by direct DMA, whereas in the system ROCm 7.2
// runtime an explicit hipMemcpyDeviceToHost into hipHostMalloc memory took 166 us for 1.8 MB
// (40 us with hipMemcpyDefault) and ran at half the rate at 256 MiB; uploads are the same
// either way (components.flux_calculator_amd/bench/dma_probe.hip, profiles/r05/dma2/).
constexpr hipMemcpyKind kH2D = hipMemcpyDefault, kD2H = hipMemcpyDefault;

// cells [a, z) of a mirror <-> the same cells of its host array.  Tiled: the whole tiles in
// between as one 2-D copy (rows = tiles), the partial head / tail tiles as 1-D copies.
static hipError_t copy_cells(const fcx_engine *e, const Buffer &bf, int64_t a, int64_t z, bool h2d,
                             hipStream_t s) {
  const size_t es = e->esize;
  auto one = [&](int64_t lo, int64_t hi) {
    if (hi <= lo) return hipSuccess;
    char *dev = reinterpret_cast<char *>(bf.dev) + (size_t)tiled(lo, e->tpad) * es;
    char *host = reinterpret_cast<char *>(bf.host) + (size_t)lo * es;
    const size_t bytes = (size_t)(hi - lo) * es;
    return h2d ? hipMemcpyAsync(dev, host, bytes, kH2D, s) : hipMemcpyAsync(host, dev, bytes, kD2H, s);
  };
  if (z <= a) return hipSuccess;
  if (e->tpad == 0) return one(a, z);
  const int64_t t0 = (a + kLayoutTile - 1) / kLayoutTile, t1 = z / kLayoutTile;  // whole tiles [t0, t1)
  if (t1 <= t0) {  // within one tile, or across one tile boundary
    const int64_t m = std::min(z, t0 * kLayoutTile);
    hipError_t r = one(a, m);
    return (r != hipSuccess || m >= z) ? r : one(m, z);
  }
  if (a < t0 * kLayoutTile)
    if (hipError_t r = one(a, t0 * kLayoutTile)) return r;
  const size_t row = (size_t)kLayoutTile * es, pitch = (size_t)(kLayoutTile + e->tpad) * es;
  char *dev = reinterpret_cast<char *>(bf.dev) + (size_t)t0 * pitch;
  char *host = reinterpret_cast<char *>(bf.host) + (size_t)t0 * row;
  hipError_t r = h2d ? hipMemcpy2DAsync(dev, pitch, host, row, row, (size_t)(t1 - t0), kH2D, s)
                     : hipMemcpy2DAsync(host, row, dev, pitch, row, (size_t)(t1 - t0), kD2H, s);
  if (r != hipSuccess || z == t1 * kLayoutTile) return r;
  return one(t1 * kLayoutTile, z);
}

// zero cells [0, n) of an engine buffer (a regrid destination without links)
static hipError_t zero_cells(const fcx_engine *e, double *dev, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (e->tpad == 0) return hipMemsetAsync(dev, 0, (size_t)n * e->esize, s);
  const size_t row = (size_t)kLayoutTile * e->esize, pitch = (size_t)(kLayoutTile + e->tpad) * e->esize;
  const int64_t full = n / kLayoutTile;
  if (full)
    if (hipError_t r = hipMemset2DAsync(dev, pitch, 0, row, (size_t)full, s)) return r;
  if (n > full * kLayoutTile)
    return hipMemsetAsync(reinterpret_cast<char *>(dev) + full * pitch, 0, (size_t)(n - full * kLayoutTile) * e->esize, s);
  return hipSuccess;
}

// ---- staging arena (FCX_OPT_HOST_STAGING) ---------------------------------------------
//
// Caller heap arrays (a Fortran host's ALLOCATEd local_field arrays, numpy arrays) are never
// page-locked or mapped: every transfer goes through an engine-owned page-locked image of
// the device pool that holds their mirrors, with the same bytes at the same offsets.  An
// upload copies the arrays into the image on the host (CopyPool threads), then moves each
// run of consecutive mirrors with ONE DMA (a tiled pool's run of slots is one 2-D copy over
// the tile rows, one 1-D copy when it spans whole rows); a download is the reverse, its host
// copies done once the stream has drained (fcx_synchronize).  Against one runtime copy per
// array (the pageable path, FCX_OPT_HOST_STAGING = 0) this removes ~15 of the ~17 copy calls
// of a step, whose fixed cost dominates the Baltic-size grid.

// which pool holds the mirror at device address d; sp = -1 when none with host-bound mirrors
static StageRef stage_ref(fcx_engine *e, const void *d) {
  StageRef r;
  const char *p = reinterpret_cast<const char *>(d);
  for (size_t i = 0; i < e->spools.size(); ++i) {
    const StagePool &q = e->spools[i];
    if (p >= q.dev && p < q.dev + q.bytes) {
      r.sp = (int)i;
      r.soff = (size_t)(p - q.dev);
      return r;
    }
  }
  return r;
}

// at commit: the pools of the engine's mirrors, and for every caller heap array (not
// fcx_host_malloc memory, which is copied by direct DMA, and not device or in-place memory)
// its place in them.  The host images are allocated at the first staged transfer.
static void stage_setup(fcx_engine *e) {
  if (!e->staging) return;
  const size_t es = e->esize;
  std::vector<StagePool> cand;
  for (void *p : e->tiled_pools)
    cand.push_back(StagePool{(char *)p, nullptr, e->tiled_bytes, true, (size_t)kLayoutTile * es,
                             (size_t)(kLayoutTile + e->tpad) * es});
  if (e->pool) cand.push_back(StagePool{(char *)e->pool, nullptr, e->pool_bytes, false, 0, 0});
  if (e->atm_pool) {
    const bool t = e->atm_out_tpad != 0;
    cand.push_back(StagePool{(char *)e->atm_pool, nullptr, e->atm_pool_bytes, t, t ? (size_t)kLayoutTile * es : 0,
                             t ? (size_t)(kLayoutTile + e->atm_out_tpad) * es : 0});
  }
  for (auto &rm : e->remaps)
    if (rm.pool) cand.push_back(StagePool{(char *)rm.pool, nullptr, rm.pool_bytes, false, 0, 0});
  // keep the pools some heap array's mirror lives in
  auto heap = [&](const void *host, int64_t n) { return host && !lib_block_device_ptr(host, (size_t)std::max<int64_t>(n, 1) * es); };
  std::vector<char> used(cand.size(), 0);
  auto mark = [&](const void *dev) {
    for (size_t i = 0; i < cand.size(); ++i)
      if ((const char *)dev >= cand[i].dev && (const char *)dev < cand[i].dev + cand[i].bytes) used[i] = 1;
  };
  for (auto &bf : e->bufs)
    if (!bf.external && heap(bf.host, bf.n)) mark(bf.dev);
  for (auto &f : e->atm_fields)
    if (!f.external && heap(f.out_host, e->n_atmos)) mark(f.out_dev);
  for (auto &rm : e->remaps)
    for (auto &f : rm.fields)
      if (!f.external && heap(f.out_host, rm.n_dst)) mark(f.out_dev);
  for (size_t i = 0; i < cand.size(); ++i)
    if (used[i]) e->spools.push_back(cand[i]);
  for (auto &bf : e->bufs)
    if (!bf.external && heap(bf.host, bf.n)) bf.st = stage_ref(e, bf.dev);
  for (auto &f : e->atm_fields)
    if (!f.external && heap(f.out_host, e->n_atmos)) f.st = stage_ref(e, f.out_dev);
  for (auto &rm : e->remaps)
    for (auto &f : rm.fields)
      if (!f.external && heap(f.out_host, rm.n_dst)) f.st = stage_ref(e, f.out_dev);
}

// A pool whose image cannot be page-locked (a memory-tight node) takes the direct path: its
// members' StageRefs are dropped, so they are copied one runtime copy per array from the
// caller's pageable memory, as with FCX_OPT_HOST_STAGING 0.  Applies at commit and at a lazy
// pool's first transfer alike, so no step and no per-call subroutine ever meets an
// allocation failure (the lazy path returned FCX_E_NOMEM, which stopped the
// coupled run through the Fortran drop-in).
static void stage_disable(fcx_engine *e, size_t i) {
  StagePool &p = e->spools[i];
  p.host = nullptr;
  p.disabled = true;
  auto drop = [&](StageRef &st) {
    if (st.sp == (int)i) st.sp = -1;
  };
  for (auto &bf : e->bufs) drop(bf.st);
  for (auto &f : e->atm_fields) drop(f.st);
  for (auto &rm : e->remaps)
    for (auto &f : rm.fields) drop(f.st);
}

// FCX_TEST_PIN_FAIL (tests only): 1 = every image fails at commit, as on a node out of
// lockable memory; 2 = only the lazy pools' images fail, at their first transfer
static int pin_fail_mode() {
  const char *v = std::getenv("FCX_TEST_PIN_FAIL");
  return v && (*v == '1' || *v == '2') ? *v - '0' : 0;
}

// page-lock pool i's image now (false: it could not be, and the pool is disabled)
static bool stage_pin(fcx_engine *e, size_t i, bool lazy) {
  StagePool &p = e->spools[i];
  if (p.host) return true;
  if (p.disabled) return false;
  const int inject = pin_fail_mode();
  if (!(inject == 1 || (inject == 2 && lazy)) &&
      hipHostMalloc((void **)&p.host, std::max<size_t>(p.bytes, 1), kHostPinFlags) == hipSuccess)
    return true;
  (void)hipGetLastError();
  stage_disable(e, i);
  return false;
}

// at commit: the host image of every staging pool a whole step transfers (page-locked, the
// pool's size: the pinned footprint is fcx_staging_bytes).  Pools only other calls transfer
// (eager[i] == 0: e.g. the tiled layout's pool of arrays no step reads or writes) get their
// image at their first transfer (page-locking them up front locked ~1 GB per
// 10M-cell engine that no step uses).
static void stage_alloc_all(fcx_engine *e, const std::vector<char> &eager) {
  const bool fail_all = pin_fail_mode() == 1;
  for (size_t i = 0; i < e->spools.size(); ++i) {
    if (e->spools[i].host) continue;  // (a mapped arena has its image already)
    if (i < eager.size() && !eager[i] && !fail_all) continue;  // at its first transfer
    (void)stage_pin(e, i, false);
  }
}

// before a transfer of buffers `ids` (and atmosphere / remap outputs) is put together: the
// lazy pools they use page-locked, or disabled so that those buffers take the direct path
static void stage_prepare_bufs(fcx_engine *e, const std::vector<int> &ids) {
  for (int b : ids) {
    const int sp = e->bufs[(size_t)b].st.sp;
    if (sp >= 0) (void)stage_pin(e, (size_t)sp, true);
  }
}
static void stage_prepare_outputs(fcx_engine *e) {
  for (auto &f : e->atm_fields)
    if (f.st.sp >= 0) (void)stage_pin(e, (size_t)f.st.sp, true);
  for (auto &rm : e->remaps)
    for (auto &f : rm.fields)
      if (f.st.sp >= 0) (void)stage_pin(e, (size_t)f.st.sp, true);
}

// the host images of the pools these transfers use (stage_prepare_* ran before the transfer
// list was made, so every pool in it has its image)
static int stage_alloc(fcx_engine *e, const std::vector<Xfer> &xs) {
  for (const Xfer &x : xs) {
    StagePool &p = e->spools[(size_t)x.sp];
    if (!p.host) return fail(FCX_E_STATE, "staging pool %d has no host image", x.sp);
  }
  return FCX_OK;
}

static void stage_free(fcx_engine *e) {
  for (auto &p : e->spools)
    if (p.host) (void)hipHostFree(p.host);  // (a mapped pool's image is its device buffer too)
  e->spools.clear();
  if (e->ev_stage_in) (void)hipEventDestroy(e->ev_stage_in);
  e->ev_stage_in = nullptr;
}

// host copies of elements [a, z) (z < 0: to the array's end) of every transfer, caller array
// -> arena image (gather) or back (scatter), spread over the copy threads
static void stage_copy(fcx_engine *e, const std::vector<Xfer> &xs, int64_t a, int64_t z, bool gather) {
  constexpr size_t kPiece = size_t(64) << 10;
  const size_t es = e->esize;
  std::vector<CopyJob> jobs;
  auto add = [&](char *img, char *host, size_t bytes) {
    for (size_t o = 0; o < bytes; o += kPiece) {
      const size_t b = std::min(kPiece, bytes - o);
      jobs.push_back(gather ? CopyJob{img + o, host + o, b} : CopyJob{host + o, img + o, b});
    }
  };
  for (const Xfer &x : xs) {
    const StagePool &p = e->spools[(size_t)x.sp];
    const int64_t lo = std::min(a, x.n), hi = z < 0 ? x.n : std::min(z, x.n);
    if (hi <= lo) continue;
    if (!p.tiled) {
      add(p.host + x.soff + (size_t)lo * es, x.host + (size_t)lo * es, (size_t)(hi - lo) * es);
      continue;
    }
    for (int64_t t0 = lo; t0 < hi;) {
      const int64_t row = t0 >> kLayoutShift, t1 = std::min(hi, (row + 1) << kLayoutShift);
      add(p.host + x.soff + (size_t)row * p.pitch + (size_t)(t0 - (row << kLayoutShift)) * es,
          x.host + (size_t)t0 * es, (size_t)(t1 - t0) * es);
      t0 = t1;
    }
  }
  // batches beyond the caches stream their stores (no read-for-ownership of the destination);
  // Baltic-size batches stay cache-resident and copy plainly
  size_t total = 0;
  for (const auto &j : jobs) total += j.bytes;
  CopyPool::get().run(jobs, e->host_threads > 0 ? e->host_threads : default_host_threads(), total >= (size_t(32) << 20));
}

// DMAs of elements [a, z) of the transfers' mirrors between arena and device: per pool,
// every run of consecutive mirrors in one copy.  Tiled pools: a run is adjacent slots, moved
// over the tile rows [a / tile, ceil(z / tile)) as one 2-D copy (1-D when the run is whole
// rows); plain pools: mirrors back to back (256-B aligned), whole arrays only.  A run holds
// transfer members only, so an upload never overwrites another mirror.
static hipError_t stage_dma(fcx_engine *e, std::vector<Xfer> xs, int64_t a, int64_t z, bool h2d, hipStream_t s) {
  const size_t es = e->esize;
  std::sort(xs.begin(), xs.end(), [](const Xfer &l, const Xfer &r) {
    return l.sp != r.sp ? l.sp < r.sp : l.soff < r.soff;
  });
  const hipMemcpyKind kind = h2d ? kH2D : kD2H;
  size_t i = 0;
  while (i < xs.size()) {
    const StagePool &p = e->spools[(size_t)xs[i].sp];
    size_t j = i + 1;
    int64_t hi = z < 0 ? xs[i].n : std::min(z, xs[i].n);
    if (p.mapped) {  // the kernels use the image in place
      while (j < xs.size() && xs[j].sp == xs[i].sp) ++j;
    } else if (p.tiled) {
      size_t end = xs[i].soff + p.slot;
      while (j < xs.size() && xs[j].sp == xs[i].sp && (xs[j].soff == end || xs[j].soff + p.slot == end)) {
        end = std::max(end, xs[j].soff + p.slot);
        hi = std::max(hi, z < 0 ? xs[j].n : std::min(z, xs[j].n));
        ++j;
      }
      const int64_t r0 = a >> kLayoutShift, r1 = (hi + kLayoutTile - 1) >> kLayoutShift;
      if (r1 > r0 && hi > a) {
        const size_t off = xs[i].soff + (size_t)r0 * p.pitch, width = end - xs[i].soff;
        char *d = p.dev + off, *h = p.host + off;
        hipError_t r = width == p.pitch
                           ? hipMemcpyAsync(h2d ? (void *)d : (void *)h, h2d ? (void *)h : (void *)d,
                                            (size_t)(r1 - r0) * p.pitch, kind, s)
                           : hipMemcpy2DAsync(h2d ? (void *)d : (void *)h, p.pitch, h2d ? (void *)h : (void *)d,
                                              p.pitch, width, (size_t)(r1 - r0), kind, s);
        if (r != hipSuccess) return r;
      }
    } else {
      const int64_t lo = std::min(a, xs[i].n);
      size_t end = xs[i].soff + (size_t)hi * es;
      if (a == 0 && z < 0)  // whole arrays: the next mirror starts at the 256-B aligned end
        while (j < xs.size() && xs[j].sp == xs[i].sp && xs[j].soff <= (end + 255) / 256 * 256 && xs[j].soff >= xs[i].soff) {
          end = std::max(end, xs[j].soff + (size_t)xs[j].n * es);
          ++j;
        }
      if (end > xs[i].soff + (size_t)lo * es) {
        const size_t off = xs[i].soff + (size_t)lo * es;
        hipError_t r = hipMemcpyAsync(h2d ? (void *)(p.dev + off) : (void *)(p.host + off),
                                      h2d ? (void *)(p.host + off) : (void *)(p.dev + off), end - off, kind, s);
        if (r != hipSuccess) return r;
      }
    }
    i = j;
  }
  return hipSuccess;
}

static int stage_flush(fcx_engine *e);

// upload through the arena: the previous upload's DMA must have left the image, and
// outputs still waiting for their host copies are completed first
static int stage_in(fcx_engine *e, const std::vector<Xfer> &xs, hipStream_t s) {
  if (xs.empty()) return FCX_OK;
  if (int r = stage_alloc(e, xs)) return r;
  bool mapped = false;
  for (const Xfer &x : xs) mapped = mapped || e->spools[(size_t)x.sp].mapped;
  if (!e->pending_out.empty() || mapped) {  // a mapped image is read by the kernels in place:
    HIP_TRY(hipStreamSynchronize(e->stream));  // the last launch must be done with it
    if (int r = stage_flush(e)) return r;
  }
  if (e->stage_in_live) HIP_TRY(hipEventSynchronize(e->ev_stage_in));
  stage_copy(e, xs, 0, -1, true);
  HIP_TRY(stage_dma(e, xs, 0, -1, true, s));
  if (!e->ev_stage_in) HIP_TRY(hipEventCreateWithFlags(&e->ev_stage_in, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(e->ev_stage_in, s));
  e->stage_in_live = true;
  return FCX_OK;
}

// download through the arena: the DMAs now; the host copies into the caller's arrays right
// away (the stream is waited for, so the arrays hold the outputs when fcx_download returns),
// or with FCX_OPT_DEFERRED_SCATTER at the next fcx_synchronize
static int stage_out(fcx_engine *e, const std::vector<Xfer> &xs, hipStream_t s) {
  if (xs.empty()) return FCX_OK;
  if (int r = stage_alloc(e, xs)) return r;
  HIP_TRY(stage_dma(e, xs, 0, -1, false, s));
  e->pending_out.insert(e->pending_out.end(), xs.begin(), xs.end());
  if (!e->deferred_scatter) {
    HIP_TRY(hipStreamSynchronize(s));
    return stage_flush(e);
  }
  return FCX_OK;
}

// after the stream has drained: the pending downloads into the caller's arrays
static int stage_flush(fcx_engine *e) {
  if (e->pending_out.empty()) return FCX_OK;
  stage_copy(e, e->pending_out, 0, -1, false);
  e->pending_out.clear();
  return FCX_OK;
}

static Xfer xfer_of(const StageRef &st, void *host, int64_t n) {
  return Xfer{st.sp, st.soff, reinterpret_cast<char *>(host), n};
}

// Zero-copy for caller heap arrays (FCX_OPT_ZERO_COPY with staging): their images live in
// one device-mapped page-locked arena (plain layout, 256-B aligned) that the kernels use in
// place -- the library's own memory, as fcx_host_malloc blocks are -- so a small step makes
// no copy call at all: the host copies the inputs into the arena, the launch reads and
// writes it over the host link, the host copies the outputs back after the synchronisation.
static int map_staged(fcx_engine *e, int *count) {
  *count = 0;
  const size_t es = e->esize;
  auto heap = [&](const void *h, int64_t n) { return h && !lib_block_device_ptr(h, (size_t)std::max<int64_t>(n, 1) * es); };
  auto span = [&](int64_t n) { return ((size_t)std::max<int64_t>(n, 1) * es + 255) / 256 * 256; };
  struct Item {
    double **dev;
    bool *ext;
    StageRef *st;
    int64_t n;
    size_t off;
  };
  std::vector<Item> items;
  size_t total = 0;
  auto add = [&](double **dev, bool *ext, StageRef *st, int64_t n) {
    items.push_back(Item{dev, ext, st, n, total});
    total += span(n);
  };
  for (auto &bf : e->bufs)
    if (!bf.external && heap(bf.host, bf.n)) add(&bf.dev, &bf.external, &bf.st, bf.n);
  for (auto &f : e->atm_fields)
    if (!f.external && heap(f.out_host, e->n_atmos)) add(&f.out_dev, &f.external, &f.st, std::max<int64_t>(e->n_atmos, 0));
  for (auto &rm : e->remaps)
    for (auto &f : rm.fields)
      if (!f.external && heap(f.out_host, rm.n_dst)) add(&f.out_dev, &f.external, &f.st, rm.n_dst);
  if (items.empty()) return FCX_OK;
  StagePool p;
  void *h = nullptr, *d = nullptr;
  hipError_t err = hipHostMalloc(&h, total, hipHostMallocMapped | kHostPinFlags);
  if (err != hipSuccess) return fail(FCX_E_NOMEM, "hipHostMalloc(%zu) for the mapped staging arena: %s", total, hipGetErrorString(err));
  err = hipHostGetDevicePointer(&d, h, 0);
  if (err != hipSuccess || !d) {
    (void)hipHostFree(h);
    return fail(FCX_E_HIP, "hipHostGetDevicePointer: %s", hipGetErrorString(err));
  }
  p.dev = reinterpret_cast<char *>(d);
  p.host = reinterpret_cast<char *>(h);
  p.bytes = total;
  p.mapped = true;
  const int sp = (int)e->spools.size();
  e->spools.push_back(p);
  for (const Item &it : items) {
    *it.dev = reinterpret_cast<double *>(p.dev + it.off);
    *it.ext = true;  // no engine mirror: the kernels use the image
    it.st->sp = sp;
    it.st->soff = it.off;
    e->zc_bytes += it.n * (int64_t)es;
  }
  for (auto &bf : e->bufs)
    if (bf.st.sp == sp) bf.in_place = true;
  *count = (int)items.size();
  return FCX_OK;
}

extern "C" int fcx_set_precision(fcx_engine *e, int precision) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if (precision != FCX_PRECISION_F64 && precision != FCX_PRECISION_F32)
    return fail(FCX_E_ARG, "precision %d unknown", precision);
  e->f32 = precision == FCX_PRECISION_F32;
  e->esize = e->f32 ? sizeof(float) : sizeof(double);
  return FCX_OK;
}

// a remap launch of nf fields gathers packed records (FCX_OPT_REMAP_PACK).  Auto: two
// fields or more, on a scattered map.  Measured (components.flux_calculator_amd/bench/
// remap_bench.py, 10M cells, 6 fields): the shuffled 2-link map (scatter 0.66) 1.46 ms from
// the arrays, 0.68 ms packed; the 1-link synthetic (0.32) 0.356 / 0.405 ms and the
// geometric map (0.31) 0.20 / 0.36 ms, where neighbouring links share their lines anyway.
constexpr double kPackScatter = 0.5;
static bool remap_packs(const fcx_engine *e, const fcx_engine::Remap &rm, int nf) {
  if (nf <= 0 || rm.n_links <= 0) return false;
  return e->remap_pack == 1 || (e->remap_pack == 2 && nf >= 2 && rm.scatter > kPackScatter);
}

// elements per packed record of nf fields: a whole number of 16-B vectors (A/B builds
// with FCX_REC_POW2: a power of two, so that no record straddles a 64-B boundary)
static int rec_width(const fcx_engine *e, int nf) {
  const int v = (int)(16 / e->esize);
#if defined(FCX_REC_POW2) && FCX_REC_POW2
  int p = v;
  while (p < nf) p *= 2;
  return p;
#else
  return (nf + v - 1) / v * v;
#endif
}

// distinct 64-B field segments per link over a sample of 256-destination blocks
static double remap_scatter(const fcx_engine::Remap &rm) {
  const int64_t nb = (rm.n_dst + 255) / 256;
  if (nb == 0 || rm.n_links == 0) return 0.0;
  const int64_t every = std::max<int64_t>(1, nb / 256);
  int64_t links = 0, distinct = 0;
  std::vector<int32_t> seg;
  for (int64_t b = 0; b < nb; b += every) {
    const int32_t k0 = rm.row[(size_t)(b * 256)], k1 = rm.row[(size_t)std::min<int64_t>(rm.n_dst, (b + 1) * 256)];
    seg.clear();
    for (int32_t k = k0; k < k1; ++k) seg.push_back(rm.col[(size_t)k] >> 3);
    std::sort(seg.begin(), seg.end());
    distinct += std::unique(seg.begin(), seg.end()) - seg.begin();
    links += k1 - k0;
  }
  return links ? (double)distinct / (double)links : 0.0;
}

extern "C" int fcx_commit(fcx_engine *e) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return FCX_OK;
  if (int r = validate(e)) return r;
  if (int r = gpu_init(e)) return r;
  // Zero-copy of fcx_host_malloc arrays.  2 (auto, default): where the pipelined step would
  // not apply (grids below two chunks, where the step is latency-bound and per-array copies
  // dominate it); 1: at any size; 0: never.  Caller heap arrays always take mirrors.
  const int64_t n_big = std::max(e->n[0], std::max(e->n[1], e->n[2]));
  const bool small = n_big < 2 * e->min_chunk;
  if (e->zero_copy == 1 || (e->zero_copy == 2 && small)) {
    // fcx_host_malloc arrays in place.  (Round 6 measured the span transport against it at
    // the Baltic size: 335-338 against 213-233 us for the three variants -- every copy and
    // launch on a stream costs ~10-17 us of dispatch latency in this runtime, which the
    // copy engines' duplex does not win back at 1-3 MB per engine)
    e->zc_active = map_host_arrays(e) > 0;
    int staged = 0;
    if (e->staging)
      if (int r = map_staged(e, &staged)) return r;
    e->zc_active = e->zc_active || staged > 0;
  }
  if (e->lib_spans) {
    int spanned = 0;
    if (int r = map_lib_spans(e, &spanned)) return r;
  }
  classify_written(e);
  bool any_external = false;
  for (auto &bf : e->bufs) any_external = any_external || bf.external;
  if (e->tiled_opt && !any_external && !e->bufs.empty()) {
    if (int r = alloc_tiled(e)) return r;
  } else {
    e->tpad = 0;
  }
  // plain layout: one pooled allocation for all host-bound mirrors, 256-B aligned sub-buffers
  size_t total = 0;
  std::vector<size_t> off(e->bufs.size(), 0);
  for (size_t b = 0; b < e->bufs.size() && e->tiled_pools.empty(); ++b) {
    if (e->bufs[b].external) continue;
    off[b] = total;
    total += ((size_t)e->bufs[b].n * e->esize + 255) / 256 * 256;
  }
  if (total) {
    e->pool_bytes = total;
    hipError_t err = hipMalloc(&e->pool, total);
    if (err != hipSuccess)
      return fail(FCX_E_NOMEM, "hipMalloc(%zu) for the field mirrors: %s", total, hipGetErrorString(err));
    for (size_t b = 0; b < e->bufs.size(); ++b)
      if (!e->bufs[b].external) e->bufs[b].dev = reinterpret_cast<double *>((char *)e->pool + off[b]);
  }
  if (e->lcorr) {
    HIP_TRY(hipMalloc(&e->corr_dev, std::max<size_t>(e->corr_mm.size(), 1) * e->esize));
    if (e->f32) {  // rounded once; the fp32 kernels add them in fp32
      std::vector<float> cf(e->corr_mm.begin(), e->corr_mm.end());
      HIP_TRY(hipMemcpy(e->corr_dev, cf.data(), cf.size() * sizeof(float), hipMemcpyHostToDevice));
    } else {
      HIP_TRY(hipMemcpy(e->corr_dev, e->corr_mm.data(), e->corr_mm.size() * sizeof(double),
                        hipMemcpyHostToDevice));
    }
  }
  for (auto &c : e->rg) {
    if (!c.set) continue;
    HIP_TRY(hipMalloc(&c.d_row, c.row_ptr.size() * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&c.d_col, std::max<size_t>(c.col.size(), 1) * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&c.d_w, std::max<size_t>(c.w.size(), 1) * sizeof(double)));
    HIP_TRY(hipMemcpy(c.d_row, c.row_ptr.data(), c.row_ptr.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    if (!c.col.empty()) {
      HIP_TRY(hipMemcpy(c.d_col, c.col.data(), c.col.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      if (e->f32) {  // REAL(wp) weights of the single-precision build: rounded once
        std::vector<float> wf(c.w.begin(), c.w.end());
        HIP_TRY(hipMemcpy(c.d_w, wf.data(), wf.size() * sizeof(float), hipMemcpyHostToDevice));
      } else {
        HIP_TRY(hipMemcpy(c.d_w, c.w.data(), c.w.size() * sizeof(double), hipMemcpyHostToDevice));
      }
    }
  }
  if (e->n_atmos >= 0) {
    HIP_TRY(hipMalloc(&e->d_atm_row, e->atm_row.size() * sizeof(int32_t)));
    HIP_TRY(hipMemcpy(e->d_atm_row, e->atm_row.data(), e->atm_row.size() * sizeof(int32_t),
                      hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&e->d_atm_w, std::max<size_t>(e->atm_w.size(), 1) * sizeof(double)));
    if (!e->atm_w.empty())
      HIP_TRY(hipMemcpy(e->d_atm_w, e->atm_w.data(), e->atm_w.size() * sizeof(double), hipMemcpyHostToDevice));
    // the per-cell index, where some fp64 launch reads it
    if (e->atm_contiguous && !e->atm_idx.empty() && !(compact_map(e->f32, true) && compact_map(e->f32, false))) {
      HIP_TRY(hipMalloc(&e->d_atm_idx, e->atm_idx.size() * sizeof(int32_t)));
      HIP_TRY(hipMemcpy(e->d_atm_idx, e->atm_idx.data(), e->atm_idx.size() * sizeof(int32_t),
                        hipMemcpyHostToDevice));
    }
    // the compacted map, where some launch reads it
    if (e->atm_contiguous && !e->atm_idx.empty() && (compact_map(e->f32, true) || compact_map(e->f32, false))) {
      const int64_t nx = (int64_t)e->atm_idx.size(), nw = (nx + 31) / 32;
      std::vector<uint32_t> seg((size_t)(2 * nw + 1), 0u);  // bits, then prefix counts (int32)
      std::vector<int32_t> atm;
      for (int64_t x = 0; x < nx; ++x)
        if (x == 0 || e->atm_idx[(size_t)x] != e->atm_idx[(size_t)x - 1]) {
          seg[(size_t)(x >> 5)] |= 1u << (x & 31);
          atm.push_back(e->atm_idx[(size_t)x]);
        }
      int32_t run = 0;
      for (int64_t w = 0; w <= nw; ++w) {
        seg[(size_t)(nw + w)] = (uint32_t)run;
        if (w < nw) run += __builtin_popcount(seg[(size_t)w]);
      }
      e->atm_seg_words = nw;
      e->atm_segments = (int64_t)atm.size();
      const size_t head = seg.size() * sizeof(uint32_t);
      HIP_TRY(hipMalloc(&e->d_atm_seg, head + std::max<size_t>(atm.size(), 1) * sizeof(int32_t)));
      HIP_TRY(hipMemcpy(e->d_atm_seg, seg.data(), head, hipMemcpyHostToDevice));
      if (!atm.empty())
        HIP_TRY(hipMemcpy((char *)e->d_atm_seg + head, atm.data(), atm.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      // the first cell's atmosphere cell of every wave tile: the crossing records' entry, where
      // launches with records read the compacted map
      if (compact_map(e->f32, false)) {
        const int64_t tc = (int64_t)(e->f32 ? kF32Cpl : 2) * 64, nt = (nx + tc - 1) / tc;
        std::vector<int32_t> a0((size_t)nt);
        for (int64_t t = 0; t < nt; ++t) a0[(size_t)t] = e->atm_idx[(size_t)(t * tc)];
        HIP_TRY(hipMalloc(&e->d_atm_tile_a0, (size_t)std::max<int64_t>(nt, 1) * sizeof(int32_t)));
        if (nt) HIP_TRY(hipMemcpy(e->d_atm_tile_a0, a0.data(), a0.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      }
    }
    if (e->atm_contiguous && !e->atm_idx.empty()) {  // the fused path's crossing records
      const int64_t tiles = (e->n[0] + kTile - 1) / kTile;
      HIP_TRY(hipMalloc(&e->d_atm_xrec, (size_t)std::max<int64_t>(tiles, 1) * kXRec * sizeof(double)));
      // tile boundaries a segment runs across: none (a map whose runs never cross a wave
      // tile) means no fix-up launch at all
      e->atm_crossings = 0;
      for (size_t b = kTile; b < e->atm_idx.size(); b += kTile) e->atm_crossings += e->atm_idx[b - 1] == e->atm_idx[b];
      if (!e->atm_empty.empty()) {
        HIP_TRY(hipMalloc(&e->d_atm_empty, e->atm_empty.size() * sizeof(int32_t)));
        HIP_TRY(hipMemcpy(e->d_atm_empty, e->atm_empty.data(), e->atm_empty.size() * sizeof(int32_t),
                          hipMemcpyHostToDevice));
      }
    }
    if (!e->atm_contiguous) {
      HIP_TRY(hipMalloc(&e->d_atm_col, std::max<size_t>(e->atm_col.size(), 1) * sizeof(int32_t)));
      if (!e->atm_col.empty())
        HIP_TRY(hipMemcpy(e->d_atm_col, e->atm_col.data(), e->atm_col.size() * sizeof(int32_t),
                          hipMemcpyHostToDevice));
    }
    size_t need = 0;
    bool atm_ext = false;
    for (auto &f : e->atm_fields) {
      atm_ext = atm_ext || f.external;
      if (!f.external) need += ((size_t)std::max<int64_t>(e->n_atmos, 1) * e->esize + 255) / 256 * 256;
    }
    // tile-blocked outputs (with the field mirrors, FCX_TILED_ATM): the fields' tiles of 4096
    // atmosphere cells side by side, so the fused kernel's segment-end stores of a wave land
    // in one region instead of one per field
    const int64_t nfa = (int64_t)e->atm_fields.size();
    if (FCX_TILED_ATM && e->tpad && !atm_ext && nfa >= 2 && e->n_atmos > 0) {
      const int64_t tiles = (e->n_atmos + kLayoutTile - 1) / kLayoutTile;
      e->atm_pool_bytes = (size_t)tiles * nfa * kLayoutTile * e->esize;
      HIP_TRY(hipMalloc(&e->atm_pool, e->atm_pool_bytes));
      for (int64_t k = 0; k < nfa; ++k)
        e->atm_fields[k].out_dev = reinterpret_cast<double *>((char *)e->atm_pool + (size_t)k * kLayoutTile * e->esize);
      e->atm_out_tpad = (nfa - 1) * kLayoutTile;
      need = 0;
    }
    if (need) {
      e->atm_pool_bytes = need;
      HIP_TRY(hipMalloc(&e->atm_pool, need));
      size_t off = 0;
      for (auto &f : e->atm_fields)
        if (!f.external) {
          f.out_dev = reinterpret_cast<double *>((char *)e->atm_pool + off);
          off += ((size_t)std::max<int64_t>(e->n_atmos, 1) * e->esize + 255) / 256 * 256;
        }
    }
  }
  if (e->own_shared && e->n_atmos >= 0) {  // [n_boundaries][fields] slots, zero on entry
    const size_t stride = std::max<size_t>(e->atm_fields.size(), 1);
    const size_t cnt = std::max<size_t>((size_t)e->atm_nb * stride, 1);
    HIP_TRY(hipMalloc(&e->atm_shared_own, cnt * sizeof(double)));
    HIP_TRY(hipMemset(e->atm_shared_own, 0, cnt * sizeof(double)));
    if (e->atm_left >= 0 && e->atm_right >= 0 && e->n_atmos < 2 && e->atm_left != e->atm_right)
      return fail(FCX_E_ARG, "the one atmosphere cell is shared on both sides: it needs one boundary slot for all "
                             "its ranks (left == right), not %d and %d", e->atm_left, e->atm_right);
    e->atm_shared = e->atm_nb > 0 ? e->atm_shared_own : nullptr;
    e->atm_stride = (int32_t)stride;
  }
  for (auto &rm : e->remaps) {
    for (auto &f : rm.fields)
      if (rm.max_src >= e->n[f.g - 1])
        return fail(FCX_E_ARG, "remap link source %d outside the %lld cells of grid %d", rm.max_src,
                    (long long)e->n[f.g - 1], f.g);
    HIP_TRY(hipMalloc(&rm.d_row, rm.row.size() * sizeof(int32_t)));
    HIP_TRY(hipMemcpy(rm.d_row, rm.row.data(), rm.row.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&rm.d_col, std::max<size_t>(rm.col.size(), 1) * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&rm.d_w, std::max<size_t>(rm.w.size(), 1) * sizeof(double)));
    if (!rm.col.empty()) {
      HIP_TRY(hipMemcpy(rm.d_col, rm.col.data(), rm.col.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(rm.d_w, rm.w.data(), rm.w.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    const size_t one = ((size_t)std::max<int64_t>(rm.n_dst, 1) * e->esize + 255) / 256 * 256;
    size_t need = 0;
    for (auto &f : rm.fields) need += f.external ? 0 : one;
    if (need) {
      rm.pool_bytes = need;
      HIP_TRY(hipMalloc(&rm.pool, need));
      size_t off = 0;
      for (auto &f : rm.fields)
        if (!f.external) {
          f.out_dev = reinterpret_cast<double *>((char *)rm.pool + off);
          off += one;
        }
    }
    // records scratch for the packed gather: the largest launch group of any phase
    size_t nf_max = 0;
    for (int ph = 1; ph <= 3; ++ph) {
      size_t c = 0;
      for (auto &f : rm.fields) c += (f.phase & ph) ? 1 : 0;
      nf_max = std::max(nf_max, std::min<size_t>(c, kMaxAtmosFields));
    }
    rm.scatter = remap_scatter(rm);
    if (remap_packs(e, rm, (int)nf_max))
      e->rec_bytes = std::max(e->rec_bytes, (size_t)(rm.max_src + 1) * rec_width(e, (int)nf_max) * e->esize);
  }
  if (e->rec_bytes) HIP_TRY(hipMalloc(&e->d_rec, e->rec_bytes));
  stage_setup(e);
  e->committed = true;
  // the pools a whole step transfers are page-locked now, the others at first use
  std::vector<char> eager(e->spools.size(), e->any_regrid ? 1 : 0);
  if (!e->any_regrid) {
    Plan *pl = nullptr;
    if (get_plan(e, phase_stages(FCX_PHASE_ALL), FCX_PHASE_ALL, &pl) == FCX_OK && pl) {
      for (const std::vector<int> *ids : {&pl->reads, &pl->writes})
        for (int b : *ids)
          if (e->bufs[(size_t)b].st.sp >= 0) eager[(size_t)e->bufs[(size_t)b].st.sp] = 1;
    } else {
      std::fill(eager.begin(), eager.end(), 1);
    }
    for (auto &f : e->atm_fields)
      if (f.st.sp >= 0) eager[(size_t)f.st.sp] = 1;
    for (auto &rm : e->remaps)
      for (auto &f : rm.fields)
        if (f.st.sp >= 0) eager[(size_t)f.st.sp] = 1;
  }
  stage_alloc_all(e, eager);
  return FCX_OK;
}

// ------------------------------------------------------------------ execution

static const uint32_t kEarly = S_RBBR;
static const uint32_t kNormal = S_QSUR_T | S_QSUR_U | S_QSUR_V | S_MEVA | S_HLAT | S_HSEN | S_UMOM |
                                S_VMOM | S_RSDR;

static int uploader_join(fcx_engine *e);

// every call but fcx_upload_field first waits for the fields fcx_upload_field handed over
static int check(fcx_engine *e) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (!e->committed) return fail(FCX_E_STATE, "fcx_commit has not been called");
  return uploader_join(e);
}

static const double *month_slice(fcx_engine *e, int32_t t, int *rc) {
  *rc = FCX_OK;
  if (!e->lcorr) return nullptr;
  int32_t m = 0;
  if ((*rc = fcx_current_month(e->init_date, t, &m)) != FCX_OK) return nullptr;
  return reinterpret_cast<const double *>((const char *)e->corr_dev + (size_t)(m - 1) * e->n[0] * e->esize);
}

// the mirrors of buffers `ids` <-> their host arrays on the engine stream: caller heap arrays
// through the staging arena, fcx_host_malloc arrays (and staging off) by direct copies
static int copy_bufs(fcx_engine *e, const std::vector<int> &ids, bool h2d, std::vector<Xfer> *more = nullptr) {
  stage_prepare_bufs(e, ids);
  std::vector<Xfer> xs;
  if (more) xs.swap(*more);
  std::vector<int> spanned;
  bool direct = false;
  for (int b : ids) {
    const Buffer &bf = e->bufs[b];
    if (bf.n == 0) continue;
    if (h2d && (size_t)b < e->field_sent.size() && e->field_sent[(size_t)b]) continue;  // fcx_upload_field
    if (bf.st.sp >= 0) {  // (also a heap array whose mirror is a mapped arena image)
      xs.push_back(xfer_of(bf.st, bf.host, bf.n));
      continue;
    }
    if (bf.span >= 0) {
      spanned.push_back(b);
      continue;
    }
    if (bf.external) continue;
    HIP_TRY(copy_cells(e, bf, 0, bf.n, h2d, e->stream));
    direct = true;
  }
  if (!spanned.empty()) {
    if (int r = span_copy(e, spanned, h2d, e->stream)) return r;
    direct = true;
  }
  if (h2d) return stage_in(e, xs, e->stream);
  if (xs.empty() && direct && !e->deferred_scatter) {  // the outputs in the arrays on return
    HIP_TRY(hipStreamSynchronize(e->stream));
    return stage_flush(e);
  }
  return stage_out(e, xs, e->stream);
}

#ifndef FCX_ZC_ONE_CELL  // A/B builds: 0 keeps 16-B (2-cell) lanes in zero-copy launches
#define FCX_ZC_ONE_CELL 1
#endif

// halo lanes of a fused launch of plan pl over the whole grid (0: crossing records and the
// fix-up launch): one surface type, on a map whose segments are short enough that `halo`
// lanes of the next tile's head (at most 1/16 of a wave) cover every crossing
static int full_range_halo(const fcx_engine *e, const Plan *pl) {
  const int cpl = e->f32 ? kF32Cpl : 2;
  const int h = (e->atm_maxseg - 1 + cpl - 1) / cpl;
  if (e->atm_halo && e->atm_crossings > 0 &&
      (pl->host.num_types == 1 || (FCX_HALO_RAVG && pl->host.ravg_on)) && h >= 1 && h <= (cpl == 4 ? 2 : 4))
    return h;
  return 0;
}

// the launch shape of plan pl over cells [lo, hi) (hi < 0: to the end); *fused: the
// exchange -> atmosphere accumulation rides in the launch (pl->af is brought up to date)
static LaunchConfig plan_launch(fcx_engine *e, Plan *pl, int64_t lo, int64_t hi, bool *fused) {
  LaunchConfig lc = e->launch;
  lc.lo = lo;
  lc.hi = hi;
  // host-mapped fields: plain loads and stores (the non-temporal hint is for HBM streams;
  // over the host link it buys nothing, and plain stores are the well-trodden path)
  if (e->zc_active) lc.nontemporal = false;
  if (!e->aligned16) lc.cells_per_thread = 1;
  // host-mapped fields (small grids): loads over the host link want many requests in flight,
  // so the grid-stride kernel runs one cell per lane (twice the waves: 32,768 cells are 512
  // waves), unless this launch also feeds the fused accumulation or writes remap records
  // (both 2 cells per lane).  Kernel 80.5 -> 72.6-75.2 us per CCLM step at 32,768 cells
  // (profiles/r03/zc_shape_ab/; one-wave workgroups on top changed nothing)
  if (FCX_ZC_ONE_CELL && e->zc_active && !pl->atm_fused && pl->host.rec == nullptr) lc.cells_per_thread = 1;
  lc.merged = pl->host.merged_uv != 0;
  lc.variant = (e->specialize && lc.merged) ? pl->variant : 0;
  lc.f32 = e->f32;
  lc.ravg = pl->host.ravg_on != 0;
  // remap records only from the T=1 specialised fp64 kernels with two cells per lane (the
  // rule plan_fused_records applied when it built the plan)
  lc.rec = pl->host.rec != nullptr && lc.variant && lc.cells_per_thread == 2 && !lc.f32;
  *fused = pl->atm_fused && lc.variant && lc.cells_per_thread == 2;
  if (*fused) {  // the shared-slot pointers may have been set after the plan was built
    pl->af.shared = e->atm_shared;
    pl->af.stride = e->atm_stride;
    pl->af.left = e->atm_left;
    pl->af.right = e->atm_right;
    // halo tiles instead of crossing records + fix-up: a launch over the whole grid (not a
    // pipelined chunk)
    lc.halo = lo == 0 && (hi < 0 || hi >= pl->host.n_max) ? full_range_halo(e, pl) : 0;
    pl->af.halo = lc.halo;
  }
  return lc;
}

// the crossing records' fix-up after a fused launch over the whole grid without halo tiles
static int launch_empty_cells(fcx_engine *e, Plan *pl, const LaunchConfig &lc) {
  if (e->atm_empty.empty()) return FCX_OK;
  const int r = launch_atmos_zero(pl->af, e->d_atm_empty, (int64_t)e->atm_empty.size(), lc.f32, e->stream);
  if (r) return fail(FCX_E_HIP, "atmos_zero launch: %s", hipGetErrorString((hipError_t)r));
  return FCX_OK;
}

static int launch_fixup(fcx_engine *e, Plan *pl, const LaunchConfig &lc) {
  if (int r = launch_empty_cells(e, pl, lc)) return r;
  if (e->atm_crossings <= 0 || lc.halo) return FCX_OK;
  const int r = launch_atmos_fixup(pl->af, pl->host.n_max, lc.f32, e->stream);
  if (r) return fail(FCX_E_HIP, "atmos_fixup launch: %s", hipGetErrorString((hipError_t)r));
  return FCX_OK;
}

static int launch_plan(fcx_engine *e, Plan *pl, const double *corr_m, int64_t lo = 0, int64_t hi = -1,
                       bool fixup = true) {
  if (pl->host.n_max <= 0) return FCX_OK;
  bool fused = false;
  const LaunchConfig lc = plan_launch(e, pl, lo, hi, &fused);
  e->rec_written = lc.rec;
  const int r = launch_cells(&pl->host, pl->dev, corr_m, lc, e->stream, fused ? &pl->af : nullptr);
  if (r) return fail(FCX_E_HIP, "cells_kernel launch: %s", hipGetErrorString((hipError_t)r));
  if (fused && fixup)
    if (int r2 = launch_fixup(e, pl, lc)) return r2;
  if (fused) e->atm_done_fused = true;
  return FCX_OK;
}

static int regrid_var(fcx_engine *e, int var, int surface_type);
static int comm_exchange(fcx_engine *e);
static hipError_t get_atm(const fcx_engine *e, double *host, const double *dev, hipStream_t s);
static int run_remaps(fcx_engine *e, int phase);
static int download_remaps(fcx_engine *e, int phase, hipStream_t s, std::vector<Xfer> *xs);

// the reference step order with do_regridding after each calc (flux_calculator.F90:972-991)
static int staged_sequence(int phase, std::vector<std::pair<uint32_t, int>> &seq) {
  if (phase & FCX_PHASE_EARLY) seq.push_back({S_RBBR, FCX_RBBR});
  if (phase & FCX_PHASE_NORMAL) {
    seq.push_back({S_QSUR_T | S_QSUR_U | S_QSUR_V, FCX_QSUR});
    seq.push_back({S_MEVA, FCX_MEVA});
    seq.push_back({S_HLAT, FCX_HLAT});
    seq.push_back({S_HSEN, FCX_HSEN});
    seq.push_back({S_UMOM, FCX_UMOM});
    seq.push_back({S_VMOM, FCX_VMOM});
    seq.push_back({S_RSDR, 0});
  }
  return FCX_OK;
}

static uint32_t phase_stages(int phase) {
  uint32_t st = S_AVG;
  if (phase & FCX_PHASE_EARLY) st |= kEarly;
  if (phase & FCX_PHASE_NORMAL) st |= kNormal;
  return st;
}

// ---- fcx_upload_field: the inputs of a phase handed over one at a time

// one field: its heap array into the arena and the DMA to its mirror (or its direct copy) on
// the engine stream -- stage_in for one buffer, on the uploader thread
static int upload_one(fcx_engine *e, int b) {
  FieldUploader &u = *e->uploader;
  const Buffer &bf = e->bufs[(size_t)b];
  if (bf.n == 0) return FCX_OK;
  if (bf.st.sp >= 0) (void)stage_pin(e, (size_t)bf.st.sp, true);  // (else: the direct path below)
  if (bf.st.sp >= 0) {
    if (!u.prepared) {  // stage_in's waits, once per step
      bool mapped = false;
      for (const StagePool &p : e->spools) mapped = mapped || p.mapped;
      if (!e->pending_out.empty() || mapped) {
        HIP_TRY(hipStreamSynchronize(e->stream));
        if (int r = stage_flush(e)) return r;
      }
      if (e->stage_in_live) HIP_TRY(hipEventSynchronize(e->ev_stage_in));
      u.prepared = true;
    }
    const std::vector<Xfer> xs{xfer_of(bf.st, bf.host, bf.n)};
    if (int r = stage_alloc(e, xs)) return r;
    stage_copy(e, xs, 0, -1, true);
    if (!e->spools[(size_t)bf.st.sp].mapped) {
      HIP_TRY(stage_dma(e, xs, 0, -1, true, e->stream));
      u.dma = true;
    }
  } else if (!bf.external || bf.span >= 0) {
    HIP_TRY(copy_cells(e, bf, 0, bf.n, true, e->stream));
  }
  return FCX_OK;
}

static void uploader_loop(fcx_engine *e) {
  FieldUploader &u = *e->uploader;
  (void)hipSetDevice(e->device);
  std::unique_lock<std::mutex> lk(u.mu);
  for (;;) {
    u.cv.wait(lk, [&] { return u.stop || !u.q.empty(); });
    if (u.q.empty()) return;  // stop
    const int b = u.q.front();
    u.q.pop_front();
    u.busy = 1;
    lk.unlock();
    const int r = upload_one(e, b);
    lk.lock();
    if (r && !u.err) {
      u.err = r;
      u.msg = g_err;
    }
    u.busy = 0;
    if (u.q.empty()) u.idle.notify_all();
  }
}

// the handed-over fields are staged and their DMAs queued (before anything else runs)
static int uploader_join(fcx_engine *e) {
  if (!e->uploader) return FCX_OK;
  FieldUploader &u = *e->uploader;
  std::unique_lock<std::mutex> lk(u.mu);
  u.idle.wait(lk, [&] { return u.q.empty() && u.busy == 0; });
  if (u.dma) {  // the next upload into the arena waits for these DMAs (stage_in's rule)
    u.dma = false;
    if (!e->ev_stage_in) HIP_TRY(hipEventCreateWithFlags(&e->ev_stage_in, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(e->ev_stage_in, e->stream));
    e->stage_in_live = true;
  }
  if (u.err) {
    const int r = u.err;
    u.err = 0;
    //  the failed hand-over leaves no field marked as sent: a host that retries
    // the step moves every input again instead of running on a stale device mirror
    std::fill(e->field_sent.begin(), e->field_sent.end(), 0);
    u.prepared = false;
    return fail(r, "fcx_upload_field: %s", u.msg.c_str());
  }
  return FCX_OK;
}

static void uploader_stop(fcx_engine *e) {
  if (!e->uploader) return;
  {
    std::lock_guard<std::mutex> lk(e->uploader->mu);
    e->uploader->stop = true;
  }
  e->uploader->cv.notify_all();
  if (e->uploader->th.joinable()) e->uploader->th.join();
  e->uploader.reset();
}

// a run takes the handed-over fields: the next step's fields start afresh
static void fields_taken(fcx_engine *e) {
  std::fill(e->field_sent.begin(), e->field_sent.end(), 0);
  if (e->uploader) e->uploader->prepared = false;  // (joined: the thread is idle)
}

extern "C" int fcx_upload_field(fcx_engine *e, int s, int g, int var) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (!e->committed) return fail(FCX_E_STATE, "fcx_commit has not been called");
  if (s < 0 || s > kMaxTypes || g < 1 || g > 3 || var < 1 || var > kNumVars)
    return fail(FCX_E_ARG, "field (%d, %d, %d) outside the data model", s, g, var);
  const int b = e->buf(s, g, var);
  if (b < 0) return fail(FCX_E_ARG, "local_field(%d,%d)%%var(%s) is not bound", s, g, kVarNames[var - 1]);
  if (e->field_sent.size() != e->bufs.size()) e->field_sent.assign(e->bufs.size(), 0);
  if (e->field_sent[(size_t)b]) return FCX_OK;  // an alias of a field already handed over
  e->field_sent[(size_t)b] = 1;
  if (!e->uploader) {
    e->uploader.reset(new FieldUploader());
    e->uploader->th = std::thread(uploader_loop, e);
  }
  {
    std::lock_guard<std::mutex> lk(e->uploader->mu);
    e->uploader->q.push_back(b);
  }
  e->uploader->cv.notify_one();
  return FCX_OK;
}

extern "C" int fcx_upload(fcx_engine *e, int phase) {
  if (int r = check(e)) return r;
  if (phase < 1 || phase > 3) return fail(FCX_E_ARG, "phase %d unknown", phase);
  Plan *pl;
  if (int r = get_plan(e, phase_stages(phase), phase, &pl)) return r;
  return copy_bufs(e, pl->reads, true);
}

extern "C" int fcx_download(fcx_engine *e, int phase) {
  if (int r = check(e)) return r;
  if (phase < 1 || phase > 3) return fail(FCX_E_ARG, "phase %d unknown", phase);
  Plan *pl;
  if (int r = get_plan(e, phase_stages(phase), phase, &pl)) return r;
  stage_prepare_outputs(e);
  std::vector<Xfer> xs;  // every staged download of the phase in one set of DMAs
  std::vector<int> ids = pl->writes;
  for (auto &f : e->atm_fields)
    if ((f.phase & phase) && e->n_atmos > 0) {
      if (f.st.sp >= 0)
        xs.push_back(xfer_of(f.st, f.out_host, e->n_atmos));
      else if (!f.external)
        HIP_TRY(get_atm(e, f.out_host, f.out_dev, e->stream));
    }
  if (int r = download_remaps(e, phase, e->stream, &xs)) return r;
  if (e->any_regrid) {  // device-side regrid destinations of the fields this phase computes
    std::vector<int> extra;
    std::vector<int> vars;
    if (phase & FCX_PHASE_EARLY) vars = {FCX_RBBR};
    if (phase & FCX_PHASE_NORMAL)
      for (int v : {FCX_QSUR, FCX_MEVA, FCX_HLAT, FCX_HSEN, FCX_UMOM, FCX_VMOM}) vars.push_back(v);
    for (int s = 1; s <= e->T; ++s)
      for (int g = 1; g <= 3; ++g)
        for (int v : vars)
          if (e->put_to[s][g - 1][v - 1])
            for (int k = 0; k < 3; ++k)
              if ((e->put_to[s][g - 1][v - 1] >> k) & 1)
                if (e->buf(s, k + 1, v) >= 0) extra.push_back(e->buf(s, k + 1, v));
    ids.insert(ids.end(), extra.begin(), extra.end());
  }
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  return copy_bufs(e, ids, false, &xs);
}

// an atmosphere output mirror -> its host array (2-D copy of the whole tiles when tiled)
static hipError_t get_atm(const fcx_engine *e, double *host, const double *dev, hipStream_t s) {
  const size_t es = e->esize, n = (size_t)e->n_atmos;
  if (!e->atm_out_tpad) return hipMemcpyAsync(host, dev, n * es, kD2H, s);
  const size_t row = (size_t)kLayoutTile * es, pitch = (size_t)(kLayoutTile + e->atm_out_tpad) * es;
  const size_t full = n / kLayoutTile;
  if (full)
    if (hipError_t r = hipMemcpy2DAsync(host, row, dev, pitch, row, full, kD2H, s)) return r;
  if (n > full * kLayoutTile)
    return hipMemcpyAsync((char *)host + full * row, (const char *)dev + full * pitch, (n - full * kLayoutTile) * es,
                          kD2H, s);
  return hipSuccess;
}

static AtmosArgs atmos_args(fcx_engine *e, int phase) {
  AtmosArgs a{};
  a.f32 = e->f32 ? 1 : 0;
  a.row_ptr = e->d_atm_row;
  a.col = e->atm_contiguous ? nullptr : e->d_atm_col;
  a.w = e->d_atm_w;
  a.n_atmos = e->n_atmos;
  a.stride = e->atm_stride;
  a.left = e->atm_left;
  a.right = e->atm_right;
  a.shared = e->atm_shared;
  a.tpad = e->tpad;
  a.out_tpad = e->atm_out_tpad;
  a.vec = a.col == nullptr && e->aligned16;
  for (size_t i = 0; i < e->atm_fields.size(); ++i) {
    const auto &f = e->atm_fields[i];
    if (!(f.phase & phase) || a.nf >= kMaxAtmosFields) continue;
    a.x[a.nf] = e->dptr(f.s, f.g, f.var);
    a.out[a.nf] = f.out_dev;
    a.scol[a.nf] = (int32_t)i;
    ++a.nf;
  }
  return a;
}

static int run_atmos(fcx_engine *e, int phase) {
  if (e->n_atmos < 0 || e->atm_fields.empty()) return FCX_OK;
  const AtmosArgs a = atmos_args(e, phase);
  if (a.nf == 0) return FCX_OK;
  const int r = launch_atmos(a, e->stream);
  if (r) return fail(FCX_E_HIP, "atmos_kernel launch: %s", hipGetErrorString((hipError_t)r));
  return FCX_OK;
}

// out[d] = sum over the links of d (link order, from 0.0) of w * field[src]: the SCRIP
// weight application OASIS performs on 'S' fields sent to a model; atmos_kernel with the
// target's CSR (columns = exchange cells), up to kMaxAtmosFields fields per launch
static int run_remaps(fcx_engine *e, int phase) {
  for (size_t ri = 0; ri < e->remaps.size(); ++ri) {
    auto &rm = e->remaps[ri];
    int gi = 0;
    AtmosArgs a{};
    a.f32 = e->f32 ? 1 : 0;
    a.row_ptr = rm.d_row;
    a.col = rm.d_col;
    a.w = rm.d_w;
    a.n_atmos = rm.n_dst;
    a.left = a.right = -1;
    a.tpad = e->tpad;
    auto flush = [&]() -> int {
      if (!a.nf) return FCX_OK;
      a.rec = nullptr;
      a.rec_p = 0;
      const Plan *rp = e->rec_plan;
      if (rp && rp->rec_remap == (int)ri && rp->rec_group == gi) {  // records written by the flux launch
        a.rec = rp->host.rec;
        a.rec_p = rp->host.rec_p;
      } else if (e->d_rec && remap_packs(e, rm, a.nf)) {  // fields -> one record per cell, then the gather
        a.rec_p = rec_width(e, a.nf);
        const int r = launch_pack_records(a, (int64_t)rm.max_src + 1, e->aligned16, !e->zc_active && e->launch.nontemporal,
                                          e->d_rec, e->stream);
        if (r) return fail(FCX_E_HIP, "remap pack launch: %s", hipGetErrorString((hipError_t)r));
        a.rec = e->d_rec;
      }
      const int r = launch_atmos(a, e->stream);
      if (r) return fail(FCX_E_HIP, "remap launch: %s", hipGetErrorString((hipError_t)r));
      a.nf = 0;
      ++gi;
      return FCX_OK;
    };
    for (auto &f : rm.fields) {
      if (!(f.phase & phase)) continue;
      a.x[a.nf] = e->dptr(f.s, f.g, f.var);
      a.out[a.nf] = f.out_dev;
      if (!a.x[a.nf]) return fail(FCX_E_MISSING, "remap field %s(%d) is not bound", kVarNames[var0(f.var)], f.s);
      if (++a.nf == kMaxAtmosFields)
        if (int r = flush()) return r;
    }
    if (int r = flush()) return r;
  }
  return FCX_OK;
}

// remap outputs -> host: staged ones appended to xs, the others copied directly
static int download_remaps(fcx_engine *e, int phase, hipStream_t s, std::vector<Xfer> *xs) {
  for (auto &rm : e->remaps)
    for (auto &f : rm.fields)
      if ((f.phase & phase) && rm.n_dst > 0) {
        if (f.st.sp >= 0)
          xs->push_back(xfer_of(f.st, f.out_host, rm.n_dst));
        else if (!f.external)
          HIP_TRY(hipMemcpyAsync(f.out_host, f.out_dev, rm.n_dst * e->esize, kD2H, s));
      }
  return FCX_OK;
}

// after the flux launch(es) of fcx_run: the accumulation when it is not fused, the boundary
// exchange of an attached communicator, the remaps, the closing timing event
static int run_tail(fcx_engine *e, int phase) {
  if (e->atmos_in_run && !e->atm_done_fused)
    if (int r = run_atmos(e, phase)) return r;
  e->atm_done = e->atmos_in_run || e->atm_done_fused;
  if (e->atm_done)
    if (int r = comm_exchange(e)) return r;
  if (int r = run_remaps(e, phase)) return r;
  if (e->timing) HIP_TRY(hipEventRecord(e->ev1, e->stream));
  e->timed = e->timing;
  return FCX_OK;
}

extern "C" int fcx_run(fcx_engine *e, int phase, int32_t t) {
  if (int r = check(e)) return r;
  if (phase < 1 || phase > 3) return fail(FCX_E_ARG, "phase %d unknown", phase);
  int rc;
  const double *corr_m = month_slice(e, t, &rc);
  if (rc) return rc;
  if (e->timing) HIP_TRY(hipEventRecord(e->ev0, e->stream));
  e->atm_done_fused = false;
  e->atm_done = e->exchanged = false;
  e->rec_plan = nullptr;
  e->group_members = 0;
  fields_taken(e);
  if (!e->any_regrid) {
    Plan *pl;
    if (int r = get_plan(e, phase_stages(phase), phase, &pl)) return r;
    if (int r = launch_plan(e, pl, corr_m)) return r;
    e->rec_plan = e->rec_written ? pl : nullptr;  // run_remaps gathers the records it wrote
  } else {
    std::vector<std::pair<uint32_t, int>> seq;
    staged_sequence(phase, seq);
    for (auto &st : seq) {
      Plan *pl;
      if (int r = get_plan(e, st.first, 0, &pl)) return r;
      if (int r = launch_plan(e, pl, corr_m)) return r;
      if (st.second)
        if (int r = regrid_var(e, st.second, 0)) return r;
    }
    Plan *pl;
    if (int r = get_plan(e, S_AVG, phase, &pl)) return r;
    if (int r = launch_plan(e, pl, nullptr)) return r;
  }
  return run_tail(e, phase);
}

struct GroupLaunchMember {
  fcx_engine *e;
  Plan *pl;
  LaunchConfig lc;
  const double *corr_m;
};
static int launch_group(const GroupLaunchMember *mem, int nm);

// the engines of a list that can share one merged launch (fcx_run_group's rule): member_of[i]
// = their index in mem, -1 for the engines that run as fcx_run.  A single one is kept.
static int select_group(fcx_engine *const *es, int n, int phase, int32_t t, std::vector<GroupLaunchMember> &mem,
                        std::vector<int> &member_of) {
  mem.clear();
  member_of.assign((size_t)n, -1);
  for (int i = 0; i < n; ++i) {
    fcx_engine *e = es[i];
    bool ok = !e->any_regrid && !e->timing && (int)mem.size() < kMaxGroup;
    GroupLaunchMember m{e, nullptr, {}, nullptr};
    if (ok) {
      int rc;
      m.corr_m = month_slice(e, t, &rc);
      if (rc) return rc;
      if (int r = get_plan(e, phase_stages(phase), phase, &m.pl)) return r;
      bool fused = false;
      m.lc = plan_launch(e, m.pl, 0, -1, &fused);
      // one surface type, or several with the type-0 averages in registers (fp64, no halo)
      const bool shape = m.pl->host.num_types == 1 || (m.lc.ravg && !m.lc.f32 && m.lc.halo == 0);
      ok = fused && shape && m.lc.variant >= 1 && !m.lc.rec && m.lc.max_blocks <= 0 && m.pl->host.n_max > 0;
      if (ok && !mem.empty()) {
        const GroupLaunchMember &f = mem[0];
        ok = e->stream == f.e->stream && e->device == f.e->device && m.lc.f32 == f.lc.f32 &&
             m.lc.nontemporal == f.lc.nontemporal && (m.lc.halo > 0) == (f.lc.halo > 0) &&
             m.lc.ravg == f.lc.ravg && (m.pl->host.num_types == 1) == (f.pl->host.num_types == 1);
      }
    }
    if (ok) {
      member_of[(size_t)i] = (int)mem.size();
      mem.push_back(m);
    }
  }
  return FCX_OK;
}

// fcx_run of several engines (e.g. one per bottom-model variant) in the order given, with
// the flux passes of those whose whole phase is one fused T = 1 launch of the same shape on
// the same stream merged into ONE launch (cells_atmos_group_kernel).  Each engine then does
// what follows its launch in fcx_run (fix-up, accumulation, exchange, remaps).  The others
// run as fcx_run.  Same results, bit for bit, as fcx_run of each.
extern "C" int fcx_run_group(fcx_engine *const *es, int n, int phase, int32_t t) {
  if (n < 0 || (n > 0 && !es)) return fail(FCX_E_ARG, "bad engine list");
  if (phase < 1 || phase > 3) return fail(FCX_E_ARG, "phase %d unknown", phase);
  for (int i = 0; i < n; ++i)
    if (int r = check(es[i])) return r;
  std::vector<GroupLaunchMember> mem;
  std::vector<int> member_of;  // list position -> member index (-1: runs as fcx_run)
  if (int r = select_group(es, n, phase, t, mem, member_of)) return r;
  if (mem.size() == 1) {  // nothing to merge
    std::fill(member_of.begin(), member_of.end(), -1);
    mem.clear();
  }
  // every engine's tail (fix-up, accumulation, boundary exchange of an attached communicator,
  // remaps) runs in LIST order below, whichever engines could join: group eligibility is
  // rank-local (map, grid cap, halo), the order of the per-engine all-reduces must not be
  if (!mem.empty())
    if (int r = launch_group(mem.data(), (int)mem.size())) return r;
  for (int i = 0; i < n; ++i) {
    fcx_engine *e = es[i];
    if (member_of[(size_t)i] < 0) {
      if (int r = fcx_run(e, phase, t)) return r;
      continue;
    }
    e->group_members = (int)mem.size();
    e->atm_done_fused = true;
    if (int r = run_tail(e, phase)) return r;
  }
  return FCX_OK;
}

// the members' group arguments (af.n_tiles: each member's tile count) and their run state reset
static void group_members(const GroupLaunchMember *mem, int nm, GroupMember *gm) {
  for (int k = 0; k < nm; ++k) {
    const GroupLaunchMember &m = mem[k];
    fcx_engine *e = m.e;
    e->atm_done_fused = false;
    e->atm_done = e->exchanged = false;
    e->rec_plan = nullptr;
    e->rec_written = false;
    fields_taken(e);
    const int64_t own = (m.lc.f32 ? kF32Cpl : 2) * (64 - m.lc.halo);
    gm[k] = GroupMember{m.pl->dev, m.corr_m, 0, m.lc.variant, 0, m.pl->af};
    gm[k].af.n_tiles = (m.pl->host.n_max + own - 1) / own;
  }
}

// the merged launch of fcx_run_group's members, their crossing-record fix-ups as one launch
// and their empty-cell stores (what precedes run_tail in fcx_run)
static int launch_group(const GroupLaunchMember *mem, int nm) {
  GroupMember gm[kMaxGroup];
  group_members(mem, nm, gm);
  const int r = launch_cells_group(gm, nm, mem[0].lc, mem[0].e->stream);
  if (r) return fail(FCX_E_HIP, "cells_atmos_group_kernel launch: %s", hipGetErrorString((hipError_t)r));
  // the members' crossing-record fix-ups (launch_fixup's rule) as one launch
  AtmosFused fx[kMaxGroup];
  int64_t fx_n[kMaxGroup];
  int nfx = 0;
#ifdef FCX_AB_BUILD
  if (mem[0].e->ab_fixup_each) {
    for (int k = 0; k < nm; ++k)
      if (int r2 = launch_fixup(mem[k].e, mem[k].pl, mem[k].lc)) return r2;
    return FCX_OK;
  }
#endif
  for (int k = 0; k < nm; ++k) {
    const GroupLaunchMember &m = mem[k];
    if (m.e->atm_crossings > 0 && m.lc.halo == 0) {
      fx[nfx] = m.pl->af;
      fx_n[nfx++] = m.pl->host.n_max;
    }
  }
  if (nfx) {
    const int r2 = launch_atmos_fixup_group(fx, fx_n, nfx, mem[0].lc.f32, mem[0].e->stream);
    if (r2) return fail(FCX_E_HIP, "atmos_fixup_group launch: %s", hipGetErrorString((hipError_t)r2));
  }
  for (int k = 0; k < nm; ++k)
    if (int r2 = launch_empty_cells(mem[k].e, mem[k].pl, mem[k].lc)) return r2;
  return FCX_OK;
}

// copy the part [lo, hi) of a host-bound buffer (the last chunk also takes the array tail)
static int copy_slice(fcx_engine *e, const Buffer &bf, int64_t lo, int64_t hi, bool last, bool h2d,
                      hipStream_t s) {
  if ((bf.external && bf.span < 0) || bf.n == 0) return FCX_OK;
  const int64_t a = std::min(lo, bf.n), z = last ? bf.n : std::min(hi, bf.n);
  if (z <= a) return FCX_OK;
  HIP_TRY(copy_cells(e, bf, a, z, h2d, s));
  return FCX_OK;
}

// fcx_step of a host-bound engine as a 3-stage pipeline over cell chunks: H2D of chunk k+1
// (s_in), the cells kernel of chunk k (engine stream) and D2H of chunk k-1 (s_out) overlap,
// so a step costs ~max(H2D bytes, D2H bytes) / link rate instead of their sum plus compute.
// Caller heap arrays go through the staging arena: this thread copies chunk k into it before
// its DMA is queued, and copies chunk k-2 out once its DMA has landed, while the copy
// engines move the chunks in between.  The accumulation fix-up / separate kernel and the
// atmosphere outputs follow the last chunk.
static int step_pipelined(fcx_engine *e, int phase, int32_t t, Plan *pl) {
  int rc;
  const double *corr_m = month_slice(e, t, &rc);
  if (rc) return rc;
  const int64_t n = pl->host.n_max;
  // chunks of at least kMinChunk cells: a chunk costs one copy call per array and one launch,
  // which only pays off once the chunk's copies are well above the call latency
  const int64_t want = std::max<int64_t>((n + e->chunks - 1) / e->chunks, e->min_chunk);
  // whole layout tiles per chunk when tiled: each array's chunk copy is one 2-D copy
  const int64_t align = e->tpad ? kLayoutTile : kChunkAlign;
  const int64_t per = (want + align - 1) / align * align;
  const int K = (int)((n + per - 1) / per);
  // the copy streams exist only for engines that take this path: every stream is a
  // hardware-queue claim (GPU_MAX_HW_QUEUES), and device-resident engines never need them
  if (!e->s_in) HIP_TRY(hipStreamCreateWithFlags(&e->s_in, hipStreamNonBlocking));
  if (!e->s_out) HIP_TRY(hipStreamCreateWithFlags(&e->s_out, hipStreamNonBlocking));
  while ((int)e->ev_in.size() < K) {
    hipEvent_t a, b, c;
    HIP_TRY(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c, hipEventDisableTiming));
    e->ev_in.push_back(a);
    e->ev_comp.push_back(b);
    e->ev_out.push_back(c);
  }
  // staged (caller heap) and direct (library memory) transfers
  stage_prepare_bufs(e, pl->reads);
  stage_prepare_bufs(e, pl->writes);
  stage_prepare_outputs(e);
  std::vector<Xfer> xin, xout;
  std::vector<int> din, dout;
  for (int b : pl->reads) {
    const Buffer &bf = e->bufs[b];
    if (bf.n == 0) continue;
    if (bf.st.sp >= 0) xin.push_back(xfer_of(bf.st, bf.host, bf.n));
    else if (!bf.external || bf.span >= 0) din.push_back(b);
  }
  for (int b : pl->writes) {
    const Buffer &bf = e->bufs[b];
    if (bf.n == 0) continue;
    if (bf.st.sp >= 0) xout.push_back(xfer_of(bf.st, bf.host, bf.n));
    else if (!bf.external || bf.span >= 0) dout.push_back(b);
  }
  if (!xin.empty() || !xout.empty()) {
    if (int r = stage_alloc(e, xin)) return r;
    if (int r = stage_alloc(e, xout)) return r;
    bool mapped = false;  // (FCX_OPT_ZERO_COPY = 1 on a large grid: the kernels read the arena)
    for (const Xfer &x : xin) mapped = mapped || e->spools[(size_t)x.sp].mapped;
    if (!e->pending_out.empty() || mapped) {  // earlier downloads still owe their host copies,
      HIP_TRY(hipStreamSynchronize(e->stream));  // or an earlier launch may still read the image
      if (int r = stage_flush(e)) return r;
    }
    if (e->stage_in_live) HIP_TRY(hipEventSynchronize(e->ev_stage_in));
  }
  auto range = [&](int k, int64_t *lo, int64_t *hi) {  // the last chunk takes the arrays' tails
    *lo = k * per;
    *hi = k == K - 1 ? -1 : std::min(n, *lo + per);
  };
  int scattered = 0;  // chunks whose outputs are in the caller's arrays
  auto scatter_upto = [&](int k_end) -> int {
    for (; scattered < k_end; ++scattered) {
      int64_t lo, hi;
      range(scattered, &lo, &hi);
      HIP_TRY(hipEventSynchronize(e->ev_out[scattered]));
      stage_copy(e, xout, lo, hi, false);
    }
    return FCX_OK;
  };
  if (e->timing) HIP_TRY(hipEventRecord(e->ev0, e->s_in));
  e->atm_done_fused = false;
  e->atm_done = e->exchanged = false;
  e->rec_plan = pl;
  for (int k = 0; k < K; ++k) {
    const int64_t lo = k * per, hi = std::min(n, lo + per);
    const bool last = k == K - 1;
    if (!xin.empty()) {
      stage_copy(e, xin, lo, last ? -1 : hi, true);
      HIP_TRY(stage_dma(e, xin, lo, last ? -1 : hi, true, e->s_in));
    }
    for (int b : din)
      if (int r = copy_slice(e, e->bufs[b], lo, hi, last, true, e->s_in)) return r;
    HIP_TRY(hipEventRecord(e->ev_in[k], e->s_in));
    HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_in[k], 0));
    if (int r = launch_plan(e, pl, corr_m, lo, hi, last)) return r;
    if (!e->rec_written) e->rec_plan = nullptr;
    HIP_TRY(hipEventRecord(e->ev_comp[k], e->stream));
    HIP_TRY(hipStreamWaitEvent(e->s_out, e->ev_comp[k], 0));
    if (!xout.empty()) HIP_TRY(stage_dma(e, xout, lo, last ? -1 : hi, false, e->s_out));
    for (int b : dout)
      if (int r = copy_slice(e, e->bufs[b], lo, hi, last, false, e->s_out)) return r;
    HIP_TRY(hipEventRecord(e->ev_out[k], e->s_out));
    if (!xout.empty() && k >= 2)
      if (int r = scatter_upto(k - 1)) return r;  // chunk k-2 has had two chunks' time to land
  }
  if (e->atmos_in_run && !e->atm_done_fused)
    if (int r = run_atmos(e, phase)) return r;
  e->atm_done = e->atmos_in_run || e->atm_done_fused;
  if (e->atm_done)
    if (int r = comm_exchange(e)) return r;
  if (int r = run_remaps(e, phase)) return r;
  HIP_TRY(hipEventRecord(e->ev_comp[K - 1], e->stream));
  HIP_TRY(hipStreamWaitEvent(e->s_out, e->ev_comp[K - 1], 0));
  std::vector<Xfer> xa;  // atmosphere and remap outputs
  if (e->atmos_in_run || e->atm_done_fused)
    for (auto &f : e->atm_fields)
      if ((f.phase & phase) && e->n_atmos > 0) {
        if (f.st.sp >= 0)
          xa.push_back(xfer_of(f.st, f.out_host, e->n_atmos));
        else if (!f.external)
          HIP_TRY(get_atm(e, f.out_host, f.out_dev, e->s_out));
      }
  if (int r = download_remaps(e, phase, e->s_out, &xa)) return r;
  if (!xa.empty()) {
    if (int r = stage_alloc(e, xa)) return r;
    HIP_TRY(stage_dma(e, xa, 0, -1, false, e->s_out));
  }
  if (e->timing) HIP_TRY(hipEventRecord(e->ev1, e->s_out));
  e->timed = e->timing;
  if (!xout.empty())
    if (int r = scatter_upto(K)) return r;
  HIP_TRY(hipStreamSynchronize(e->s_out));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (!xa.empty()) stage_copy(e, xa, 0, -1, false);
  return FCX_OK;
}

static bool host_bound(const fcx_engine *e, const Plan *pl) {
  for (int b : pl->reads)
    if (!e->bufs[b].external || e->bufs[b].st.sp >= 0 || e->bufs[b].span >= 0) return true;
  for (int b : pl->writes)
    if (!e->bufs[b].external || e->bufs[b].st.sp >= 0 || e->bufs[b].span >= 0) return true;
  return false;
}

extern "C" int fcx_step(fcx_engine *e, int phase, int32_t t) {
  if (int r = check(e)) return r;
  if (phase < 1 || phase > 3) return fail(FCX_E_ARG, "phase %d unknown", phase);
  const bool handed = std::find(e->field_sent.begin(), e->field_sent.end(), 1) != e->field_sent.end();
  if (e->chunks > 1 && !e->any_regrid && !handed) {  // (fields handed over: the sequential step)
    Plan *pl;
    if (int r = get_plan(e, phase_stages(phase), phase, &pl)) return r;
    if (host_bound(e, pl) && pl->host.n_max >= 2 * e->min_chunk) return step_pipelined(e, phase, t, pl);
  }
  if (int r = fcx_upload(e, phase)) return r;
  if (int r = fcx_run(e, phase, t)) return r;
  if (int r = fcx_download(e, phase)) return r;
  return fcx_synchronize(e);
}

// fcx_step without the final wait: the inputs are in the engine's hands when it returns (caller
// heap arrays copied into the staging arena), the launch and the downloads are queued, and the
// caller's output arrays are filled by the next fcx_synchronize.  A host can start the next
// engine (or its own work: the other phase's oasis_get, diagnostics) meanwhile.  Host-bound
// grids that take the chunk pipeline complete inside the call.
extern "C" int fcx_step_async(fcx_engine *e, int phase, int32_t t) {
  if (int r = check(e)) return r;
  if (phase < 1 || phase > 3) return fail(FCX_E_ARG, "phase %d unknown", phase);
  const bool handed = std::find(e->field_sent.begin(), e->field_sent.end(), 1) != e->field_sent.end();
  if (e->chunks > 1 && !e->any_regrid && !handed) {  // (fields handed over: the sequential step)
    Plan *pl;
    if (int r = get_plan(e, phase_stages(phase), phase, &pl)) return r;
    if (host_bound(e, pl) && pl->host.n_max >= 2 * e->min_chunk) return step_pipelined(e, phase, t, pl);
  }
  if (int r = fcx_upload(e, phase)) return r;
  if (int r = fcx_run(e, phase, t)) return r;
  const bool keep = e->deferred_scatter;
  e->deferred_scatter = true;  // the host copies of the downloads wait for fcx_synchronize
  const int r = fcx_download(e, phase);
  e->deferred_scatter = keep;
  return r;
}

extern "C" int fcx_synchronize(fcx_engine *e) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed)
    if (int r = uploader_join(e)) return r;
  HIP_TRY(hipStreamSynchronize(e->stream));
  return stage_flush(e);
}

// one reference subroutine: upload what it reads, run, download what it writes
static int per_call(fcx_engine *e, uint32_t stages, int avg_phases, int32_t t) {
  if (int r = check(e)) return r;
  Plan *pl;
  if (int r = get_plan(e, stages, avg_phases, &pl)) return r;
  int rc;
  const double *corr_m = (stages & S_MEVA) ? month_slice(e, t, &rc) : nullptr;
  if ((stages & S_MEVA) && rc) return rc;
  if (int r = copy_bufs(e, pl->reads, true)) return r;
  fields_taken(e);
  if (e->timing) HIP_TRY(hipEventRecord(e->ev0, e->stream));
  if (int r = launch_plan(e, pl, corr_m)) return r;
  if (e->timing) HIP_TRY(hipEventRecord(e->ev1, e->stream));
  e->timed = e->timing;
  if (int r = copy_bufs(e, pl->writes, false)) return r;
  return fcx_synchronize(e);
}

extern "C" int fcx_calc_spec_vapor_surface(fcx_engine *e, int g) {
  if (g < 1 || g > 3) return fail(FCX_E_ARG, "which_grid %d", g);
  return per_call(e, g == 1 ? S_QSUR_T : g == 2 ? S_QSUR_U : S_QSUR_V, 0, 0);
}
extern "C" int fcx_calc_flux_mass_evap(fcx_engine *e, int32_t t) { return per_call(e, S_MEVA, 0, t); }
extern "C" int fcx_calc_flux_heat_latent(fcx_engine *e) { return per_call(e, S_HLAT, 0, 0); }
extern "C" int fcx_calc_flux_heat_sensible(fcx_engine *e) { return per_call(e, S_HSEN, 0, 0); }
extern "C" int fcx_calc_flux_momentum_east(fcx_engine *e, int g) {
  if (g != 2) return fail(FCX_E_UNSUPPORTED, "eastward momentum is computed on the u grid (2), got %d", g);
  return per_call(e, S_UMOM, 0, 0);
}
extern "C" int fcx_calc_flux_momentum_north(fcx_engine *e, int g) {
  if (g != 3) return fail(FCX_E_UNSUPPORTED, "northward momentum is computed on the v grid (3), got %d", g);
  return per_call(e, S_VMOM, 0, 0);
}
extern "C" int fcx_calc_flux_radiation_blackbody(fcx_engine *e) { return per_call(e, S_RBBR, 0, 0); }
extern "C" int fcx_distribute_shortwave_radiation_flux(fcx_engine *e) { return per_call(e, S_RSDR, 0, 0); }

extern "C" int fcx_average_across_surface_types(fcx_engine *e, int g, int var) {
  if (g < 1 || g > 3 || var < 1 || var > kNumVars) return fail(FCX_E_ARG, "bad average arguments");
  return per_call(e, S_AVG, 1000 + 100 * g + var, 0);
}

// basic:463-522 on the device buffers (dst zeroed, CSR rows in link order)
static int regrid_var(fcx_engine *e, int var, int surface_type) {
  static const int from_g[4] = {2, 3, 1, 1}, to_g[4] = {1, 1, 2, 3}, bit[4] = {1, 1, 2, 4};
  for (int s = 1; s <= kMaxTypes; ++s) {
    if (!(s == surface_type || surface_type == 0)) continue;
    for (int k = 0; k < 4; ++k) {
      if (!(e->put_to[s][from_g[k] - 1][var0(var)] & bit[k])) continue;
      const Csr &c = e->rg[k];
      double *dst = e->dptr(s, to_g[k], var);
      const double *src = e->dptr(s, from_g[k], var);
      if (!dst || !src) return fail(FCX_E_MISSING, "regridding %s: source or destination unbound", kVarNames[var0(var)]);
      if (!c.set) {
        HIP_TRY(zero_cells(e, dst, e->n[to_g[k] - 1], e->stream));
        continue;
      }
      int r = launch_regrid_csr(c.d_row, c.d_col, c.d_w, src, dst, c.n_dst, e->stream, e->f32, e->tpad);
      if (r) return fail(FCX_E_HIP, "regrid: %s", hipGetErrorString((hipError_t)r));
    }
  }
  return FCX_OK;
}

extern "C" int fcx_do_regridding(fcx_engine *e, int var, int surface_type) {
  if (int r = check(e)) return r;
  if (var < 1 || var > kNumVars || surface_type < 0 || surface_type > kMaxTypes)
    return fail(FCX_E_ARG, "bad regridding arguments");
  static const int from_g[4] = {2, 3, 1, 1}, to_g[4] = {1, 1, 2, 3}, bit[4] = {1, 1, 2, 4};
  std::vector<int> src, dst;
  for (int s = 1; s <= kMaxTypes; ++s) {
    if (!(s == surface_type || surface_type == 0)) continue;
    for (int k = 0; k < 4; ++k)
      if (e->put_to[s][from_g[k] - 1][var0(var)] & bit[k]) {
        src.push_back(e->buf(s, from_g[k], var));
        dst.push_back(e->buf(s, to_g[k], var));
      }
  }
  if (src.empty()) return FCX_OK;
  for (int b : src)
    if (b < 0) return fail(FCX_E_MISSING, "regridding %s: source unbound", kVarNames[var0(var)]);
  for (int b : dst)
    if (b < 0) return fail(FCX_E_MISSING, "regridding %s: destination unbound", kVarNames[var0(var)]);
  if (int r = copy_bufs(e, src, true)) return r;
  if (int r = regrid_var(e, var, surface_type)) return r;
  if (int r = copy_bufs(e, dst, false)) return r;
  return fcx_synchronize(e);
}

// ------------------------------------------------------------------ queries

extern "C" int fcx_device_ptr(fcx_engine *e, int s, int g, int var, double **dptr) {
  if (int r = check(e)) return r;
  if (!dptr || s < 0 || s > kMaxTypes || g < 1 || g > 3 || var < 1 || var > kNumVars)
    return fail(FCX_E_ARG, "bad arguments");
  *dptr = e->dptr(s, g, var);
  return FCX_OK;
}

extern "C" int fcx_device_layout(fcx_engine *e, int64_t *tile, int64_t *tile_stride) {
  if (int r = check(e)) return r;
  if (!tile || !tile_stride) return fail(FCX_E_ARG, "NULL argument");
  *tile = kLayoutTile;
  *tile_stride = kLayoutTile + e->tpad;
  return FCX_OK;
}

extern "C" int fcx_last_kernel_ms(fcx_engine *e, float *ms) {
  if (!e || !ms) return fail(FCX_E_ARG, "NULL argument");
  if (!e->timing) return fail(FCX_E_STATE, "timing is off: set FCX_OPT_TIMING to 1 before the run");
  if (!e->timed) return fail(FCX_E_STATE, "no run recorded");
  HIP_TRY(hipEventSynchronize(e->ev1));
  HIP_TRY(hipEventElapsedTime(ms, e->ev0, e->ev1));
  return FCX_OK;
}

extern "C" int fcx_staging_bytes(fcx_engine *e, int64_t *bytes) {
  if (int r = check(e)) return r;
  if (!bytes) return fail(FCX_E_ARG, "NULL argument");
  int64_t b = 0;
  for (auto &p : e->spools)
    if (p.host) b += (int64_t)p.bytes;  // page-locked images only (a disabled pool has none)
  *bytes = b;
  return FCX_OK;
}

// retired in version 3 (kept as stubs for one release): nothing is page-locked for the
// caller any more, and the in-launch carry hand-off and its recoveries are gone
extern "C" int fcx_pinned_bytes(fcx_engine *e, int64_t *bytes) {
  if (!e || !bytes) return fail(FCX_E_ARG, "NULL argument");
  *bytes = 0;
  return FCX_OK;
}

extern "C" int fcx_handoff_recoveries(fcx_engine *e, int64_t *count) {
  if (!e || !count) return fail(FCX_E_ARG, "NULL argument");
  *count = 0;
  return FCX_OK;
}

extern "C" int fcx_span_runs(fcx_engine *e, int phase, int32_t *h2d_copies, int32_t *d2h_copies) {
  if (int r = check(e)) return r;
  if (phase < 1 || phase > 3 || !h2d_copies || !d2h_copies) return fail(FCX_E_ARG, "bad arguments");
  Plan *pl;
  if (int r = get_plan(e, phase_stages(phase), phase, &pl)) return r;
  int n[2] = {0, 0};
  for (int k = 0; k < 2; ++k) {
    std::vector<int> ids;
    for (int b : k ? pl->writes : pl->reads)
      if (e->bufs[(size_t)b].span >= 0 && e->bufs[(size_t)b].n > 0) ids.push_back(b);
    if (int r = span_copy(e, ids, k == 0, nullptr, &n[k])) return r;
  }
  *h2d_copies = n[0];
  *d2h_copies = n[1];
  return FCX_OK;
}

extern "C" int fcx_zero_copy_bytes(fcx_engine *e, int64_t *bytes) {
  if (int r = check(e)) return r;
  if (!bytes) return fail(FCX_E_ARG, "NULL argument");
  *bytes = e->zc_bytes;
  return FCX_OK;
}

extern "C" int fcx_algorithmic_bytes(fcx_engine *e, int phase, int64_t *bytes) {
  if (int r = check(e)) return r;
  if (!bytes || phase < 1 || phase > 3) return fail(FCX_E_ARG, "bad arguments");
  Plan *pl;
  if (int r = get_plan(e, phase_stages(phase), phase, &pl)) return r;
  int64_t b = 0;
  for (int id : pl->reads) b += e->bufs[id].n;
  for (int id : pl->writes) b += e->bufs[id].n;
  if (e->lcorr && (phase & FCX_PHASE_NORMAL)) b += e->n[0];
  int64_t extra = 0;  // atmosphere accumulation: weights (+cols), re-read fields, outputs
  int nf = 0;
  for (auto &f : e->atm_fields) nf += (f.phase & phase) ? 1 : 0;
  const int64_t es = (int64_t)e->esize;
  if (pl->atm_fused && e->specialize && e->launch.cells_per_thread == 2 && e->aligned16 &&
      (!e->f32 || e->launch.max_blocks <= 0)) {
    nf = 0;  // fused: the map (compacted, or an index per cell) and a weight per cell, the
             // atmosphere outputs (fluxes not re-read)
    const bool compact = compact_map(e->f32, full_range_halo(e, pl) > 0);
    extra = e->n[0] * 8 + (compact ? (2 * e->atm_seg_words + 1 + e->atm_segments) * 4 : e->n[0] * 4) +
            (int64_t)pl->atm_nf * e->n_atmos * es;
  } else if (nf && e->n_atmos >= 0 && e->atmos_in_run) {
    extra += e->n[0] * 8 + (e->atm_contiguous ? 0 : e->n[0] * 4) + (e->n_atmos + 1) * 4;
    extra += (int64_t)nf * (e->n[0] + e->n_atmos) * es;
  }
  *bytes = b * (int64_t)e->esize + extra;
  return FCX_OK;
}

// ------------------------------------------------------------------ device memory

extern "C" int fcx_device_malloc(int device, size_t bytes, void **ptr) {
  if (!ptr) return fail(FCX_E_ARG, "ptr is NULL");
  HIP_TRY(hipSetDevice(device));
  hipError_t err = hipMalloc(ptr, bytes ? bytes : 1);
  if (err != hipSuccess) return fail(FCX_E_NOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(err));
  return FCX_OK;
}

extern "C" int fcx_device_free(void *ptr) {
  HIP_TRY(hipFree(ptr));
  return FCX_OK;
}

extern "C" int fcx_memcpy(void *dst, const void *src, size_t bytes, int kind) {
  const hipMemcpyKind k = kind == 1   ? hipMemcpyHostToDevice
                          : kind == 2 ? hipMemcpyDeviceToHost
                          : kind == 3 ? hipMemcpyDeviceToDevice
                                      : hipMemcpyDefault;
  if (kind < 1 || kind > 3) return fail(FCX_E_ARG, "memcpy kind %d", kind);
  HIP_TRY(hipMemcpy(dst, src, bytes, k));
  return FCX_OK;
}

// ------------------------------------------------------------------ tuning

// The cached plans were built for the launch options of their time (which kernel writes the
// remap records, whether the accumulation rides in the flux launch): options that change
// that drop them, and the next run builds them again.
static int drop_plans(fcx_engine *e) {
  if (e->plans.empty()) return FCX_OK;
  if (e->stream) HIP_TRY(hipStreamSynchronize(e->stream));
  for (auto &kv : e->plans) {
    (void)hipFree(kv.second.dev);
    (void)hipFree(kv.second.host.rec);
  }
  e->plans.clear();
  e->rec_plan = nullptr;
  return FCX_OK;
}

extern "C" int fcx_set_option(fcx_engine *e, int option, int64_t value) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  switch (option) {
    case FCX_OPT_CELLS_PER_THREAD:
      if (value != 1 && value != 2) return fail(FCX_E_ARG, "cells per thread must be 1 or 2");
      if (e->launch.cells_per_thread != (int)value)
        if (int r = drop_plans(e)) return r;
      e->launch.cells_per_thread = (int)value;
      return FCX_OK;
    case FCX_OPT_MAX_BLOCKS:
      if (value < -1 || value > (1 << 30)) return fail(FCX_E_ARG, "max blocks %lld", (long long)value);
      e->launch.max_blocks = (int)value;
      return FCX_OK;
    case FCX_OPT_NONTEMPORAL:
      e->launch.nontemporal = value != 0;
      return FCX_OK;
    case FCX_OPT_SPECIALIZE:
      if (e->specialize != (value != 0))
        if (int r = drop_plans(e)) return r;
      e->specialize = value != 0;
      return FCX_OK;
    case FCX_OPT_ATMOS_IN_RUN:
      e->atmos_in_run = value != 0;
      return FCX_OK;
    case FCX_OPT_TIMING:
      e->timing = value != 0;
      if (!e->timing) e->timed = false;
      return FCX_OK;
    case FCX_OPT_LIB_SPANS:
      if (e->committed) return fail(FCX_E_STATE, "lib_spans is applied at fcx_commit");
      if (value < 0 || value > 1) return fail(FCX_E_ARG, "lib_spans: 0 or 1");
      e->lib_spans = value != 0;
      return FCX_OK;
    case FCX_OPT_ZERO_COPY:
      if (e->committed) return fail(FCX_E_STATE, "zero_copy is applied at fcx_commit");
      if (value < 0 || value > 2) return fail(FCX_E_ARG, "zero_copy: 0 off, 1 on, 2 auto");
      e->zero_copy = (int)value;
      return FCX_OK;
    case FCX_OPT_PIPELINE_MIN_CHUNK:
      if (value < kChunkAlign || value % kChunkAlign)
        return fail(FCX_E_ARG, "pipeline min chunk %lld: a positive multiple of %lld cells", (long long)value,
                    (long long)kChunkAlign);
      e->min_chunk = value;
      return FCX_OK;
    case FCX_OPT_PIPELINE_CHUNKS:
      if (value < 1 || value > 1024) return fail(FCX_E_ARG, "pipeline chunks %lld outside 1..1024", (long long)value);
      e->chunks = (int)value;
      return FCX_OK;
    case FCX_OPT_ATMOS_HALO:
      e->atm_halo = value != 0;
      return FCX_OK;
    case FCX_OPT_HOST_STAGING:
      if (e->committed) return fail(FCX_E_STATE, "host_staging is applied at fcx_commit");
      e->staging = value != 0;
      return FCX_OK;
    case FCX_OPT_HOST_THREADS:
      if (value < 0 || value > 64) return fail(FCX_E_ARG, "host threads %lld outside 0..64", (long long)value);
      e->host_threads = (int)value;
      return FCX_OK;
    case FCX_OPT_REMAP_PACK:
      if (e->committed) return fail(FCX_E_STATE, "remap_pack is applied at fcx_commit");
      if (value < 0 || value > 2) return fail(FCX_E_ARG, "remap_pack: 0 never, 1 always, 2 auto");
      e->remap_pack = (int)value;
      return FCX_OK;
    case FCX_OPT_TILED_LAYOUT:
      if (e->committed) return fail(FCX_E_STATE, "tiled_layout is applied at fcx_commit");
      e->tiled_opt = value != 0;
      return FCX_OK;
    case FCX_OPT_DEFERRED_SCATTER:
      e->deferred_scatter = value != 0;
      return FCX_OK;
    case FCX_OPT_RETIRED_PIN_HOST:
    case FCX_OPT_RETIRED_12:
    case FCX_OPT_RETIRED_CARRY_HANDOFF:
      // removed in version 3 (nothing of the caller's memory is page-locked; the in-launch
      // carry hand-off is gone): accepted and ignored, so hosts that set them still run
      return FCX_OK;
#ifdef FCX_AB_BUILD
    case 98:  // measurement builds: no head records (wrong crossing values; cost of the stores)
      e->ab_no_head = value != 0;
      for (auto &kv : e->plans) kv.second.af.xrec_on = !e->ab_no_head && e->atm_crossings > 0;
      return FCX_OK;
    case 99:  // measurement builds: the group's fix-ups as one launch per member (old path)
      e->ab_fixup_each = value != 0;
      return FCX_OK;
#endif
    default:
      return fail(FCX_E_ARG, "option %d unknown", option);
  }
}

// ------------------------------------------------------------------ atmosphere accumulation

extern "C" int fcx_set_atmos_map(fcx_engine *e, int64_t n_atmos, const int32_t *idx, const double *w) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  const int64_t n = e->n[0];
  if (n_atmos < 0 || (n > 0 && (!idx || !w))) return fail(FCX_E_ARG, "bad atmosphere map");
  std::vector<int32_t> count((size_t)n_atmos + 1, 0);
  bool sorted = true;
  for (int64_t x = 0; x < n; ++x) {
    if (idx[x] < 0 || idx[x] >= n_atmos)
      return fail(FCX_E_ARG, "atmosphere index %d of exchange cell %lld outside 0..%lld", idx[x],
                  (long long)x, (long long)n_atmos - 1);
    if (x > 0 && idx[x] < idx[x - 1]) sorted = false;
    count[(size_t)idx[x] + 1]++;
  }
  e->n_atmos = n_atmos;
  e->atm_idx.assign(idx, idx + n);
  e->atm_maxseg = 0;
  e->atm_empty.clear();
  for (int64_t a = 0; a < n_atmos; ++a) {
    e->atm_maxseg = std::max(e->atm_maxseg, count[(size_t)a + 1]);
    if (count[(size_t)a + 1] == 0) e->atm_empty.push_back((int32_t)a);
  }
  e->atm_row.assign((size_t)n_atmos + 1, 0);
  for (int64_t a = 0; a < n_atmos; ++a) e->atm_row[(size_t)a + 1] = e->atm_row[(size_t)a] + count[(size_t)a + 1];
  e->atm_contiguous = sorted;
  e->atm_w.assign((size_t)n, 0.0);
  e->atm_col.clear();
  if (sorted) {
    for (int64_t x = 0; x < n; ++x) e->atm_w[(size_t)x] = w[x];
  } else {  // CSR by atmosphere cell, links kept in increasing exchange cell order
    e->atm_col.assign((size_t)n, 0);
    std::vector<int32_t> fill(e->atm_row.begin(), e->atm_row.end() - 1);
    for (int64_t x = 0; x < n; ++x) {
      const int32_t at = fill[(size_t)idx[x]]++;
      e->atm_col[(size_t)at] = (int32_t)x;
      e->atm_w[(size_t)at] = w[x];
    }
  }
  return FCX_OK;
}

extern "C" int fcx_add_atmos_field(fcx_engine *e, int phase, int s, int g, int var, double *out, int flags) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if (e->n_atmos < 0) return fail(FCX_E_STATE, "fcx_set_atmos_map first");
  if (phase < 1 || phase > 3 || s < 0 || s > kMaxTypes || g < 1 || g > 3 || var < 1 || var > kNumVars || !out)
    return fail(FCX_E_ARG, "bad atmosphere field arguments");
  if (e->n[g - 1] != e->n[0]) return fail(FCX_E_UNSUPPORTED, "atmosphere fields must live on the t grid cells");
  if ((int)e->atm_fields.size() >= kMaxAtmosFields)
    return fail(FCX_E_UNSUPPORTED, "more than %d atmosphere fields", kMaxAtmosFields);
  fcx_engine::AtmosField f;
  f.phase = phase;
  f.s = s;
  f.g = g;
  f.var = var;
  if (flags & FCX_MEM_DEVICE) {
    f.out_dev = out;
    f.external = true;
  } else {
    f.out_host = out;
  }
  e->atm_fields.push_back(f);
  return FCX_OK;
}

extern "C" int fcx_set_atmos_shared(fcx_engine *e, double *shared, int32_t nb, int32_t stride, int32_t left,
                                    int32_t right) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (nb < 0 || stride < 0 || left >= nb || right >= nb || (nb > 0 && !shared))
    return fail(FCX_E_ARG, "bad shared boundary buffer");
  if ((left >= 0 || right >= 0) && stride < (int32_t)e->atm_fields.size())
    return fail(FCX_E_ARG, "stride %d < %zu atmosphere fields", stride, e->atm_fields.size());
  if (left >= 0 && right >= 0 && e->n_atmos == 1 && left != right)
    return fail(FCX_E_ARG, "the one atmosphere cell is shared on both sides: it needs one boundary slot for all "
                           "its ranks (left == right), not %d and %d", left, right);
  if (e->own_shared) return fail(FCX_E_STATE, "boundary slots already owned by the engine (fcx_set_atmos_boundaries)");
  e->atm_shared = shared;
  e->atm_nb = nb;
  e->atm_stride = stride;
  e->atm_left = left;
  e->atm_right = right;
  return FCX_OK;
}

extern "C" int fcx_atmos_finish(fcx_engine *e) {
  if (int r = check(e)) return r;
  if (!e->atm_shared) return FCX_OK;
  if (e->n_atmos <= 0) {  // a rank without cells (io:101-104): nothing to write back, but its
                          // slots hold the reduced sums of an in-place all-reduce: re-zeroed
    if (e->atm_nb > 0 && e->atm_stride > 0)
      HIP_TRY(hipMemsetAsync(e->atm_shared, 0, (size_t)e->atm_nb * e->atm_stride * sizeof(double), e->stream));
    return FCX_OK;
  }
  const AtmosArgs a = atmos_args(e, FCX_PHASE_ALL);
  const int r = launch_atmos_finish(a, e->atm_nb, e->stream);
  if (r) return fail(FCX_E_HIP, "atmos_finish launch: %s", hipGetErrorString((hipError_t)r));
  return FCX_OK;
}

extern "C" int fcx_run_atmos(fcx_engine *e, int phase) {
  if (int r = check(e)) return r;
  if (phase < 1 || phase > 3) return fail(FCX_E_ARG, "phase %d unknown", phase);
  if (!e->atm_done) {  // not done inside the last fcx_run (FCX_OPT_ATMOS_IN_RUN = 0, not fused)
    if (int r = run_atmos(e, phase)) return r;
    e->atm_done = true;
  }
  return comm_exchange(e);  // no-op without a communicator, or when fcx_run already exchanged
}

extern "C" int fcx_last_group_size(fcx_engine *e, int32_t *members) {
  if (!e || !members) return fail(FCX_E_ARG, "NULL argument");
  *members = e->group_members;
  return FCX_OK;
}

// ------------------------------------------------------------------ exchange -> model remaps

extern "C" int fcx_add_remap(fcx_engine *e, int64_t n_dst, int64_t n_links, const int32_t *src,
                             const int32_t *dst, const double *w, int32_t *remap_id) {
  if (!e || !remap_id) return fail(FCX_E_ARG, "NULL argument");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if (n_dst < 0 || n_links < 0 || (n_links > 0 && (!src || !dst || !w))) return fail(FCX_E_ARG, "bad remap");
  fcx_engine::Remap rm;
  rm.n_dst = n_dst;
  rm.n_links = n_links;
  rm.row.assign((size_t)n_dst + 1, 0);
  for (int64_t k = 0; k < n_links; ++k) {
    if (dst[k] < 0 || dst[k] >= n_dst || src[k] < 0)
      return fail(FCX_E_ARG, "remap link %lld (%d -> %d) outside the grids", (long long)k, src[k], dst[k]);
    rm.row[(size_t)dst[k] + 1]++;
    rm.max_src = std::max(rm.max_src, src[k]);
  }
  for (int64_t d = 0; d < n_dst; ++d) rm.row[(size_t)d + 1] += rm.row[(size_t)d];
  rm.col.assign((size_t)n_links, 0);
  rm.w.assign((size_t)n_links, 0.0);
  std::vector<int32_t> fill(rm.row.begin(), rm.row.end() - 1);
  for (int64_t k = 0; k < n_links; ++k) {  // stable: each destination keeps its link order
    const int32_t at = fill[(size_t)dst[k]]++;
    rm.col[(size_t)at] = src[k];
    rm.w[(size_t)at] = w[k];
  }
  *remap_id = (int32_t)e->remaps.size();
  e->remaps.push_back(std::move(rm));
  return FCX_OK;
}

extern "C" int fcx_add_remap_field(fcx_engine *e, int32_t remap_id, int phase, int s, int g, int var, double *out,
                                   int flags) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if (remap_id < 0 || remap_id >= (int32_t)e->remaps.size()) return fail(FCX_E_ARG, "remap %d unknown", remap_id);
  if (phase < 1 || phase > 3 || s < 0 || s > kMaxTypes || g < 1 || g > 3 || var < 1 || var > kNumVars || !out)
    return fail(FCX_E_ARG, "bad remap field arguments");
  fcx_engine::RemapField f;
  f.phase = phase;
  f.s = s;
  f.g = g;
  f.var = var;
  if (flags & FCX_MEM_DEVICE) {
    f.out_dev = out;
    f.external = true;
  } else {
    f.out_host = out;
  }
  e->remaps[(size_t)remap_id].fields.push_back(f);
  return FCX_OK;
}

extern "C" int fcx_remap_info(const fcx_engine *e, int32_t remap_id, double *scatter, int32_t *packed) {
  if (!e || !scatter || !packed) return fail(FCX_E_ARG, "NULL argument");
  if (!e->committed) return fail(FCX_E_STATE, "remap info is known after fcx_commit");
  if (remap_id < 0 || remap_id >= (int32_t)e->remaps.size()) return fail(FCX_E_ARG, "remap %d unknown", remap_id);
  const auto &rm = e->remaps[(size_t)remap_id];
  int nf_max = 0;
  for (int ph = 1; ph <= 3; ++ph) {
    int c = 0;
    for (auto &f : rm.fields) c += (f.phase & ph) ? 1 : 0;
    nf_max = std::max(nf_max, std::min(c, kMaxAtmosFields));
  }
  *scatter = rm.scatter;
  *packed = e->d_rec && remap_packs(e, rm, nf_max) ? 1 : 0;
  if (e->rec_plan && e->rec_plan->rec_remap == remap_id) *packed = 2;  // the last run's flux launch wrote them
  return FCX_OK;
}

// ------------------------------------------------------------------ RCCL: the one collective
//
// The exchange -> atmosphere accumulation is the only cross-rank step of the path
// (flux_calculator.F90:1015 oasis_put of the 'S A xxxx 00' fields,
// create_namcouple.F90:92-98): the partial sums of the atmosphere cells shared by two
// neighbouring APPLE ranges are completed by ONE all-reduce (sum, fp64) of the boundary
// slots per step, over xGMI on an MI355X node.  RCCL is bound at run time (dlopen) so that
// a process that already carries an RCCL -- PyTorch-ROCm ships its own librccl.so -- uses
// that one, and a Fortran host gets /opt/rocm's; libfcx has no link-time RCCL dependency.
#include <dlfcn.h>
#include <rccl/rccl.h>

namespace {

struct RcclApi {
  bool ok = false;
  std::string why;
  ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

const RcclApi &rccl() {
  static RcclApi api = [] {
    RcclApi a;
    void *h = nullptr;
    // FCX_RCCL_LIBRARY: an explicit library with the same entry points (tests: a host-memory
    // stand-in that lets several ranks share one GPU, which RCCL refuses, and checks that every
    // rank issues the same collective sequence)
    const char *forced = std::getenv("FCX_RCCL_LIBRARY");
    if (forced && *forced) {
      h = dlopen(forced, RTLD_NOW | RTLD_LOCAL);
    } else {
      h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);  // already in the process (torch)
      if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    }
    if (!h) {
      const char *m = dlerror();
      a.why = m ? m : "librccl.so not found";
      return a;
    }
    bool all = true;
    auto sym = [&](const char *name) {
      void *p = dlsym(h, name);
      if (!p) all = false;
      return p;
    };
    a.GetUniqueId = reinterpret_cast<decltype(a.GetUniqueId)>(sym("ncclGetUniqueId"));
    a.CommInitRank = reinterpret_cast<decltype(a.CommInitRank)>(sym("ncclCommInitRank"));
    a.CommDestroy = reinterpret_cast<decltype(a.CommDestroy)>(sym("ncclCommDestroy"));
    a.AllReduce = reinterpret_cast<decltype(a.AllReduce)>(sym("ncclAllReduce"));
    a.GetErrorString = reinterpret_cast<decltype(a.GetErrorString)>(sym("ncclGetErrorString"));
    a.ok = all;
    if (!all) a.why = std::string(forced && *forced ? forced : "librccl.so") + " lacks an nccl* entry point";
    return a;
  }();
  return api;
}

#define RCCL_TRY(expr)                                                                               \
  do {                                                                                               \
    ncclResult_t r_ = (expr);                                                                        \
    if (r_ != ncclSuccess) return fail(FCX_E_HIP, "%s: %s", #expr, rccl().GetErrorString(r_));      \
  } while (0)

}  // namespace

struct fcx_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  std::vector<hipEvent_t> events;  // stream joins of fcx_atmos_allreduce (engines on several streams)
  // the boundary exchange's collective contract (atmos_exchange): packing scratch for slot
  // regions that are not one contiguous run in list order, and the exchange signature every
  // rank has agreed on (checked once per signature by a blocking max-all-reduce)
  double *scratch = nullptr;
  size_t scratch_cap = 0;
  double *agree = nullptr;  // 2 * kSigWords doubles (device)
  std::vector<double> agreed;
  bool verify_every = false;  // fcx_comm_verify: the agreement before every exchange
};

extern "C" int fcx_comm_unique_id(void *id) {
  if (!id) return fail(FCX_E_ARG, "id is NULL");
  if (!rccl().ok) return fail(FCX_E_UNSUPPORTED, "RCCL unavailable: %s", rccl().why.c_str());
  RCCL_TRY(rccl().GetUniqueId(reinterpret_cast<ncclUniqueId *>(id)));
  return FCX_OK;
}

extern "C" int fcx_comm_create(int device, int nranks, int rank, const void *id, fcx_comm **out) {
  if (!out || !id) return fail(FCX_E_ARG, "NULL argument");
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(FCX_E_ARG, "rank %d of %d", rank, nranks);
  if (!rccl().ok) return fail(FCX_E_UNSUPPORTED, "RCCL unavailable: %s", rccl().why.c_str());
  HIP_TRY(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  auto *c = new fcx_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  const ncclResult_t r = rccl().CommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(FCX_E_HIP, "ncclCommInitRank(%d of %d): %s", rank, nranks, rccl().GetErrorString(r));
  }
  *out = c;
  return FCX_OK;
}

extern "C" int fcx_comm_destroy(fcx_comm *c) {
  if (!c) return FCX_OK;
  for (hipEvent_t ev : c->events) (void)hipEventDestroy(ev);
  (void)hipFree(c->scratch);
  (void)hipFree(c->agree);
  if (c->comm) (void)rccl().CommDestroy(c->comm);
  delete c;
  return FCX_OK;
}

extern "C" int fcx_comm_allreduce_sum(fcx_comm *c, double *buf, size_t count, void *stream) {
  if (!c || (count && !buf)) return fail(FCX_E_ARG, "NULL argument");
  if (!count) return FCX_OK;
  RCCL_TRY(rccl().AllReduce(buf, buf, count, ncclFloat64, ncclSum, c->comm, reinterpret_cast<hipStream_t>(stream)));
  return FCX_OK;
}

// The boundary exchange of one or several engines of this rank: ONE all-reduce (sum, fp64)
// over the boundary slots of the listed engines, in list order, on the first engine's
// stream, then fcx_atmos_finish of each.  Engines on other streams are joined with events
// before and after.  The collective contract -- the call sequence is the same on every rank
// whatever each rank's memory layout or engine state, so no rank is left waiting:
//  * the count is sum(n_boundaries * stride) over the listed engines that have boundary
//    slots: configuration, the same on every rank of one decomposition (n_boundaries = P-1);
//  * the slots are reduced in place when the regions follow each other in list order in one
//    buffer (the bench's layout), else through the communicator's scratch (device copies each
//    way): the choice changes copies, never the collective;
//  * an engine with nothing new in its slots -- already completed in this run by its
//    attached communicator, or no accumulation since its last exchange -- takes part with
//    zeros and is not finished; the second case is an error returned AFTER the collective;
//  * the first exchange of each signature (engines with slots, values, their n_boundaries
//    and strides in order) is preceded by a blocking max-all-reduce of the signature and its
//    negation: ranks that disagree all return the same named error instead of entering
//    all-reduces of different counts (RCCL would hang).
namespace {
constexpr int kSigWords = 3;
}

static int exchange_agree(fcx_comm *c, const std::vector<double> &sig, hipStream_t s) {
  if (!c->verify_every)
    for (size_t i = 0; i + kSigWords <= c->agreed.size(); i += kSigWords)
      if (std::equal(sig.begin(), sig.end(), c->agreed.begin() + (std::ptrdiff_t)i)) return FCX_OK;
  if (!c->agree) HIP_TRY(hipMalloc(&c->agree, 2 * kSigWords * sizeof(double)));
  double h[2 * kSigWords];
  for (int i = 0; i < kSigWords; ++i) {
    h[i] = sig[(size_t)i];
    h[kSigWords + i] = -sig[(size_t)i];
  }
  HIP_TRY(hipMemcpyAsync(c->agree, h, sizeof h, hipMemcpyHostToDevice, s));
  RCCL_TRY(rccl().AllReduce(c->agree, c->agree, 2 * kSigWords, ncclFloat64, ncclMax, c->comm, s));
  HIP_TRY(hipMemcpyAsync(h, c->agree, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  bool same = true;
  for (int i = 0; i < kSigWords; ++i) same = same && h[i] == -h[kSigWords + i];
  if (!same)
    return fail(FCX_E_ARG,
                "ranks disagree on the boundary exchange (rank %d of %d): here %.0f engines with boundary slots, "
                "%.0f slot values, layout hash %.0f; over the ranks %.0f..%.0f engines, %.0f..%.0f values, hash "
                "%.0f..%.0f",
                c->rank, c->nranks, sig[0], sig[1], sig[2], -h[3], h[0], -h[4], h[1], -h[5], h[2]);
  if (!c->verify_every) c->agreed.insert(c->agreed.end(), sig.begin(), sig.end());
  return FCX_OK;
}

extern "C" int fcx_comm_verify(fcx_comm *c, int every_exchange) {
  if (!c) return fail(FCX_E_ARG, "NULL communicator");
  c->verify_every = every_exchange != 0;
  return FCX_OK;
}

static int atmos_exchange(fcx_comm *c, fcx_engine *const *es, int n) {
  std::vector<fcx_engine *> v;  // the engines with boundary slots, in list order
  for (int i = 0; i < n; ++i)
    if (es[i]->atm_shared && es[i]->atm_nb > 0 && es[i]->atm_stride > 0) v.push_back(es[i]);
  uint64_t hash = 1469598103ull;
  size_t total = 0;
  for (auto *e : v) {
    total += (size_t)e->atm_nb * e->atm_stride;
    hash = (hash * 1000003ull + (uint64_t)e->atm_nb * 4099ull + (uint64_t)e->atm_stride) & ((1ull << 48) - 1);
  }
  hipStream_t s0 = n > 0 ? es[0]->stream : nullptr;
  if (int r = exchange_agree(c, {(double)v.size(), (double)total, (double)hash}, s0)) return r;
  if (v.empty()) return FCX_OK;
  s0 = v[0]->stream;
  std::vector<char> fresh(v.size());
  int stale = -1;  // first engine with no accumulation since its last exchange
  bool inplace = true;
  for (size_t i = 0; i < v.size(); ++i) {
    fresh[i] = v[i]->atm_done && !v[i]->exchanged;
    if (!v[i]->atm_done && stale < 0) stale = (int)i;
    inplace = inplace && fresh[i] &&
              (i == 0 || v[i - 1]->atm_shared + (size_t)v[i - 1]->atm_nb * v[i - 1]->atm_stride == v[i]->atm_shared);
  }
  // the engines' streams other than the collective's, each once: a cross-stream edge costs
  // ~10 us of device time on MI355X (profiles/r05/ovprobe/), so one per stream, not per engine
  std::vector<hipStream_t> others;
  for (auto *e : v)
    if (e->stream != s0 && std::find(others.begin(), others.end(), e->stream) == others.end())
      others.push_back(e->stream);
  while (c->events.size() < 2 * others.size()) {
    hipEvent_t ev;
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    c->events.push_back(ev);
  }
  size_t k = 0;
  for (hipStream_t so : others) {  // the all-reduce waits for those engines' accumulation
    HIP_TRY(hipEventRecord(c->events[k], so));
    HIP_TRY(hipStreamWaitEvent(s0, c->events[k++], 0));
  }
  if (inplace) {
    RCCL_TRY(rccl().AllReduce(v[0]->atm_shared, v[0]->atm_shared, total, ncclFloat64, ncclSum, c->comm, s0));
  } else {
    if (c->scratch_cap < total) {
      (void)hipFree(c->scratch);
      c->scratch = nullptr;
      c->scratch_cap = 0;
      HIP_TRY(hipMalloc(&c->scratch, total * sizeof(double)));
      c->scratch_cap = total;
    }
    size_t off = 0;
    for (size_t i = 0; i < v.size(); ++i) {
      const size_t cnt = (size_t)v[i]->atm_nb * v[i]->atm_stride;
      if (fresh[i])
        HIP_TRY(hipMemcpyAsync(c->scratch + off, v[i]->atm_shared, cnt * sizeof(double), hipMemcpyDeviceToDevice, s0));
      else
        HIP_TRY(hipMemsetAsync(c->scratch + off, 0, cnt * sizeof(double), s0));
      off += cnt;
    }
    RCCL_TRY(rccl().AllReduce(c->scratch, c->scratch, total, ncclFloat64, ncclSum, c->comm, s0));
    off = 0;
    for (size_t i = 0; i < v.size(); ++i) {
      const size_t cnt = (size_t)v[i]->atm_nb * v[i]->atm_stride;
      if (fresh[i])
        HIP_TRY(hipMemcpyAsync(v[i]->atm_shared, c->scratch + off, cnt * sizeof(double), hipMemcpyDeviceToDevice, s0));
      off += cnt;
    }
  }
  for (hipStream_t so : others) {  // the finishes on that stream wait for the all-reduce
    HIP_TRY(hipEventRecord(c->events[k], s0));
    HIP_TRY(hipStreamWaitEvent(so, c->events[k++], 0));
  }
  // the finishes: the engines of one stream and precision in launches of up to kMaxGroup
  // (one block each), in list order; an engine without cells re-zeroes its slots itself
  std::vector<char> done(v.size(), 0);
  for (size_t i = 0; i < v.size(); ++i) {
    if (!fresh[i] || done[i]) continue;
    fcx_engine *e = v[i];
    if (e->n_atmos <= 0) {
      if (int r = fcx_atmos_finish(e)) return r;
      done[i] = 1;
      continue;
    }
    AtmosArgs as[kMaxGroup];
    int32_t nbs[kMaxGroup];
    int ng = 0;
    for (size_t j = i; j < v.size() && ng < kMaxGroup; ++j)
      if (fresh[j] && !done[j] && v[j]->n_atmos > 0 && v[j]->stream == e->stream && v[j]->f32 == e->f32) {
        as[ng] = atmos_args(v[j], FCX_PHASE_ALL);
        nbs[ng++] = v[j]->atm_nb;
        done[j] = 1;
      }
    const int r = launch_atmos_finish_group(as, nbs, ng, e->stream);
    if (r) return fail(FCX_E_HIP, "atmos_finish_group launch: %s", hipGetErrorString((hipError_t)r));
  }
  for (size_t i = 0; i < v.size(); ++i)
    if (fresh[i]) v[i]->exchanged = true;
  if (stale >= 0)
    return fail(FCX_E_STATE,
                "boundary exchange: engine %d of the list has no accumulation since its last exchange (fcx_run or "
                "fcx_run_atmos first); it took part with zeros",
                stale);
  return FCX_OK;
}

extern "C" int fcx_atmos_allreduce(fcx_comm *c, fcx_engine *const *engines, int n_engines) {
  if (!c || n_engines < 0 || (n_engines && !engines)) return fail(FCX_E_ARG, "bad arguments");
  for (int i = 0; i < n_engines; ++i)
    if (int r = check(engines[i])) return r;
  return atmos_exchange(c, engines, n_engines);
}

extern "C" int fcx_set_comm(fcx_engine *e, fcx_comm *c) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  e->comm = c;
  return FCX_OK;
}

// the engine's own boundary exchange after its accumulation (fcx_set_comm).  Once its slots
// are completed in this run there is nothing to agree on and nothing to send: fcx_run_atmos
// after an fcx_run that exchanged issues no collective (every rank ran the same fcx_run)
static int comm_exchange(fcx_engine *e) {
  if (!e->comm || e->exchanged) return FCX_OK;
  fcx_engine *one[1] = {e};
  return atmos_exchange(e->comm, one, 1);
}

extern "C" int fcx_set_atmos_boundaries(fcx_engine *e, int32_t n_boundaries, int32_t left, int32_t right) {
  if (!e) return fail(FCX_E_ARG, "NULL engine");
  if (e->committed) return fail(FCX_E_STATE, "engine already committed");
  if (n_boundaries < 0 || left >= n_boundaries || right >= n_boundaries || left < -1 || right < -1)
    return fail(FCX_E_ARG, "boundaries: %d slots, left %d, right %d", n_boundaries, left, right);
  e->own_shared = true;
  e->atm_nb = n_boundaries;
  e->atm_left = left;
  e->atm_right = right;
  return FCX_OK;
}
