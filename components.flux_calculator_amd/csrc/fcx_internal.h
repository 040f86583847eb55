// fcx_internal.h -- engine <-> kernel contract (device parameter block) of libfcx.
#pragma once
#include <cstdint>
#include "../../include/fcx.h"

// Measurement switches that make the kernels compute WRONG results (they take work out to
// time what is left).  They exist for the A/B builds of tools/build_variant.sh only, which
// define FCX_AB_BUILD; a product build that sets one of them does not compile.
#if !defined(FCX_AB_BUILD)
#if defined(FCX_TRIVIAL_MATH) || defined(FCX_DBG_ATM_NOLDS) || defined(FCX_DBG_ATM_NOSTORE) || \
    defined(FCX_DBG_NO_HEAD)
#error "FCX_TRIVIAL_MATH / FCX_DBG_*: wrong-result measurement builds need FCX_AB_BUILD"
#endif
#endif
#ifndef FCX_TRIVIAL_MATH  // every formula returns a plain sum of its inputs
#define FCX_TRIVIAL_MATH 0
#endif
#ifndef FCX_DBG_ATM_NOLDS  // no LDS products in the fused accumulation (sums of garbage)
#define FCX_DBG_ATM_NOLDS 0
#endif
#ifndef FCX_DBG_ATM_NOSTORE  // no atmosphere-output stores
#define FCX_DBG_ATM_NOSTORE 0
#endif
#ifndef FCX_DBG_NO_HEAD  // no crossing-record head stores
#define FCX_DBG_NO_HEAD 0
#endif
// Wave timestamps of the fused kernel (measurement builds only: correct results, but an extra
// kernel argument and a store per wave; fcx_debug_wave_trace, bench/wave_trace.py)
#if !defined(FCX_AB_BUILD) && defined(FCX_WAVE_TRACE)
#error "FCX_WAVE_TRACE is a measurement build (FCX_AB_BUILD)"
#endif
#ifndef FCX_WAVE_TRACE
#define FCX_WAVE_TRACE 0
#endif
// halo tiles also for the multi-type kernel with register averages (A/B)
#ifndef FCX_HALO_RAVG
#define FCX_HALO_RAVG 0
#endif
// the fp64 launches' exchange -> atmosphere map (fp32 launches always read the compacted
// one): 0 = a 4-B index per cell; 1 = the compacted map in halo launches, the index in
// launches with crossing records; 2 = the compacted map in every launch
#ifndef FCX_F64_COMPACT
#define FCX_F64_COMPACT 1
#endif

namespace fcx {

constexpr int kMaxTypes = FCX_MAX_SURFACE_TYPES;
constexpr int kNumVars = FCX_NUM_VARS;
constexpr int kMaxAvg = 24;

// Stage bits of one launch, in the reference call order (flux_calculator.F90:902-991).
enum Stage : uint32_t {
  S_RBBR = 1u << 0,    // calc_flux_radiation_blackbody          (early phase)
  S_QSUR_T = 1u << 1,  // calc_spec_vapor_surface(t)
  S_QSUR_U = 1u << 2,  // calc_spec_vapor_surface(u)
  S_QSUR_V = 1u << 3,  // calc_spec_vapor_surface(v)
  S_MEVA = 1u << 4,    // calc_flux_mass_evap (+ bias)
  S_HLAT = 1u << 5,    // calc_flux_heat_latent
  S_HSEN = 1u << 6,    // calc_flux_heat_sensible
  S_UMOM = 1u << 7,    // calc_flux_momentum_east  (u grid)
  S_VMOM = 1u << 8,    // calc_flux_momentum_north (v grid)
  S_RSDR = 1u << 9,    // distribute_shortwave_radiation_flux
  S_AVG = 1u << 10,    // average_across_surface_types of the registered type-0 outputs
};

// Per surface type, per launch.  A nullptr input means "not needed by this launch"; a
// nullptr output means "not stored" (method none/copy, or stage not in this launch).
struct TGridPtrs {
  const double *tsur, *fice, *psur, *patm, *qatm, *tatm, *uatm, *vatm;
  const double *amoi, *cmoi, *chea;
  const double *qsur_in;  // QSUR(s,t) when not produced in-register (none/copy/not run)
  const double *meva_in;  // MEVA(s,t) when MEVA is not produced in this launch
  double *qsur, *meva, *hlat, *hsen, *rbbr, *rsdr;
};
struct UVGridPtrs {
  const double *tsur, *fice, *psur, *uatm, *vatm, *amom, *cmom;
  const double *qsur_in;
  double *qsur, *mom;  // mom = UMOM on the u grid, VMOM on the v grid
};
struct TypeParams {
  TGridPtrs t;
  UVGridPtrs uv[2];
  int8_t m_qsur[3], m_meva, m_hlat, m_hsen, m_mom, m_rbbr;
  int8_t bias_adds;  // how many times corr(month) is added to MEVA (1 + #'copy' aliases)
  int8_t pad[7];
};
// type-0 average: X0 = sum_{s=1..T} X_s * FARE_s, in order (calc:376-383)
struct AvgEntry {
  double *x0;
  int32_t grid;  // 0,1,2
  int32_t pad;
  const double *x[kMaxTypes];
  const double *fare[kMaxTypes];
};
// Type-0 averages accumulated in registers while the surface types are processed (the
// kernel produces X_s, adds X_s * FARE_s to an accumulator, in type order from 0.0: the
// sum of calc:377-383 without re-reading X_s or FARE_s).  One slot per value the cells
// kernel holds in registers; slots 0..5 are also the fused accumulation fields.
enum AvgSlot : int { A_MEVA = 0, A_HLAT = 1, A_HSEN = 2, A_RBBR = 3, A_UMOM = 4, A_VMOM = 5, A_TSUR = 6 };
constexpr int kAvgSlots = 7;
struct AvgRegs {
  double *out[kAvgSlots];          // type-0 array of the slot, nullptr = not averaged in registers
  const double *fare[kMaxTypes];   // FARE(s) of the t grid (shared by every register slot)
};

// Tile-blocked field layout (FCX_OPT_TILED_LAYOUT).  Cell j of a field array lives at
// element (j >> kLayoutShift) * tile_stride + (j & (kLayoutTile - 1)) of its buffer; the
// kernels get tpad = tile_stride - kLayoutTile and address base + j + (j >> kLayoutShift) * tpad
// (tpad = 0: plain contiguous arrays).  Chunk boundaries of a tiled engine are whole tiles.
#ifndef FCX_LAYOUT_SHIFT  // A/B builds: tiles of 2^shift cells (4096 measured best)
#define FCX_LAYOUT_SHIFT 12
#endif
constexpr int kLayoutShift = FCX_LAYOUT_SHIFT;
constexpr int64_t kLayoutTile = int64_t(1) << kLayoutShift;
__host__ __device__ inline int64_t tiled(int64_t j, int64_t tpad) { return j + (j >> kLayoutShift) * tpad; }

struct Params {
  int64_t n[3];          // cells per grid
  int64_t n_max;         // max of the grids in this launch
  int32_t num_types;
  uint32_t stages;
  const double *rsdd0;   // RSDD of type 0 (t grid), for S_RSDR
  int32_t merged_uv;     // u/v grids are the t grid (same buffers, same sizes)
  int32_t num_avg;
  TypeParams type[kMaxTypes];
  AvgEntry avg[kMaxAvg];  // averages done by re-reading X_s (the rest)
  AvgRegs ravg;
  int32_t ravg_on;        // any ravg.out set (selects the RAVG kernel instantiation)
  int32_t pad2;
  int64_t tpad;           // tile-blocked layout of every field pointer above (0: contiguous)
  // remap records written by the T=1 specialised launch (the fields of one remap launch
  // group, fcx_engine.hip plan_fused_records): cell j's record at rec + j * rec_p, the value
  // of register slot k (AvgSlot 0..5) at position rec_pos[k] (-1 = not in the record)
  double *rec;
  int32_t rec_p;
  int8_t rec_pos[6];
  int8_t pad3[2];
};

// launchers (fcx_kernels.hip); return hipError_t as int
// how one cells_kernel launch is instantiated
struct LaunchConfig {
  int cells_per_thread = 2;  // 1 or 2 (2 needs 16-B aligned arrays)
  int max_blocks = -1;       // grid-stride cap; 0 = one unit per thread; -1 = per-kernel
                             // default (cells_kernel: 8192, fused accumulation: one trip)
  bool nontemporal = true;   // non-temporal hint on the streamed loads/stores
  bool merged = false;       // u/v grids are the t grid
  int variant = 0;           // 0 generic, 1 CCLM, 2 MOM5, 3 RCO (T=1 specialisations)
  bool f32 = false;          // fp32 fields (FCX_PRECISION_F32): 4 cells per lane
  bool ravg = false;         // register averages in this plan (Params::ravg_on)
  int64_t lo = 0, hi = -1;   // cell range of this launch (lo a multiple of kChunkAlign;
                             // hi < 0: to n_max) -- the pipelined host-bound step
  bool rec = false;          // Params::rec set: the launch also writes remap records
                             // (T=1 specialised fp64 kernels, 2 cells per lane)
  int halo = 0;              // fused accumulation with halo tiles (AtmosFused::halo lanes)
};
constexpr int64_t kChunkAlign = 1024;  // chunk boundaries: whole wave tiles and vectors

struct AtmosFused;
// corr_m: month slice [n_t] of the bias corrections (device), or nullptr
int launch_cells(const Params *host_params, const Params *dev_params, const double *corr_m,
                 const LaunchConfig &lc, void *stream, const AtmosFused *atm = nullptr);
constexpr int kMaxAtmosFields = 16;
struct AtmosArgs {
  const int32_t *row_ptr;  // [n_atmos + 1] into the exchange cells (CSR by atmosphere cell)
  const int32_t *col;      // exchange cell of each link, or nullptr when col[k] == k
  const double *w;         // [links]
  int64_t n_atmos;
  int32_t nf;
  int32_t stride;
  int32_t left, right;     // boundary slot of the first / last atmosphere cell, -1 = none
  double *shared;
  const double *x[kMaxAtmosFields];
  double *out[kMaxAtmosFields];
  int32_t f32;             // fields and outputs are float arrays (fp32 engine); the weights,
                           // products and sums stay fp64 (OASIS maps in double)
  int64_t tpad;            // layout of the x fields (engine buffers)
  int64_t out_tpad;        // layout of out: the engine's tiled atmosphere pool, or 0
  int32_t vec;             // col == nullptr and every x 16-B aligned: vector staging loads
  int32_t rec_p;           // elements per record of rec (nf rounded up to a 16-B multiple)
  const void *rec;         // remap gather: the x fields packed cell-major (pack_records),
                           // record of exchange cell j at rec + j * rec_p; nullptr = SoA gather
  int32_t scol[kMaxAtmosFields];  // column of field f in the shared boundary slots: the
                                  // field's registration index (fcx_add_atmos_field order),
                                  // the same for every phase and for the fused kernel
};
int launch_atmos(const AtmosArgs &a, void *stream);
// atmos_finish of several engines (same precision, one stream) in one launch
struct FinishGroup;
int launch_atmos_finish_group(const AtmosArgs *as, const int32_t *n_boundaries, int n, void *stream);
// remap records: rec[j * P + f] = x[f][tiled(j)] for f < nf, 0 for nf <= f < P, cells
// j < n (P a multiple of the 16-B vector length); aligned16: every x is 16-B aligned;
// nontemporal: streaming hint on the field loads (off for host-mapped fields)
int launch_pack_records(const AtmosArgs &a, int64_t n, bool aligned16, bool nontemporal, void *rec, void *stream);

// Exchange -> atmosphere accumulation fused into the T=1 cells kernel.  The six fluxes it
// can take from registers, in this order: MEVA HLAT HSEN RBBR UMOM VMOM (out[k] nullptr =
// not accumulated).  Every 128-cell wave tile sums the segments that start in it; a
// segment running past the tile end leaves its prefix sum in the next tile's crossing
// record, whose head cells atmos_fixup_kernel adds after the launch in link order (no wave
// ever waits on another).
constexpr int kFusedFields = 6;
constexpr int kRecHead = 4;     // head products kept per crossing record (longer heads: recomputed)
constexpr int kXRec = 32;       // doubles per crossing record (256 B, two lines)
constexpr int kTile = 128;  // cells per wave iteration (64 lanes x 2)
// the fused launches that read the compacted map (AtmosFused::seg_*) rather than idx
constexpr bool compact_map(bool f32, bool halo) {
  return f32 || FCX_F64_COMPACT == 2 || (FCX_F64_COMPACT == 1 && halo);
}
struct AtmosFused {
  // the exchange -> atmosphere map of a contiguous (sorted) map, compacted (round 5): bit x of
  // seg_bits[x / 32] is set where exchange cell x starts a segment (its atmosphere cell
  // differs from cell x-1's); seg_pre[w] counts the starts in cells < 32 w; seg_atm[s] is the
  // atmosphere cell of segment s.  1/8 + 1/8 + 4/(cells per segment) bytes per cell instead
  // of a 4-B index per cell.  Which launches read it and which read idx: compact_map().
  const uint32_t *seg_bits;
  const int32_t *seg_pre;
  const int32_t *seg_atm;
  const int32_t *tile_a0;  // compacted map: the atmosphere cell of each wave tile's first cell
                           // (crossing records; a load that depends on nothing)
  const int32_t *idx;  // the local atmosphere cell of every exchange cell
  const double *w;
  double *out[kFusedFields];
  const double *x[kFusedFields];  // the stored outputs (read by the fix-up only)
  double *xrec;        // [n_tiles][kXRec] crossing records (atmos_fixup_kernel):
                       // record t = the carry of tile t-1's last segment (doubles 0..5), the
                       // products w * x of tile t's first kRecHead head cells (6..29, cell-major)
                       // and {head cells, their atmosphere cell} of tile t (int2 at double 30);
                       // fp32 engines index the records by their 256-cell tiles
  int32_t xrec_on;     // some segment crosses a tile boundary: the launch fills the records
  int32_t halo;        // > 0: halo tiles (no records, no fix-up): a wave owns the cells of its
                       // first 64 - halo lanes and computes the fluxes of the last `halo`
                       // lanes' cells -- the head of the next tile -- for its products only,
                       // so every segment that starts in its own cells ends inside the wave
                       // (needs halo * C >= the longest segment - 1; full-range launches)
  int64_t n_atmos;
  double *shared;
  int32_t stride, left, right;
  int64_t tpad;        // layout of x (engine buffers); idx, w are contiguous
  int64_t out_tpad;    // layout of out (tiled atmosphere pool, or 0)
  int32_t scol[kFusedFields];  // shared-slot column of fused field k (AtmosArgs::scol)
  int64_t n_tiles;     // tiles [lo / tile cells, n_tiles) of one launch (set per launch, so no
                       // wave divides by the halo-dependent tile size)
#if FCX_WAVE_TRACE
  uint64_t *trace;     // per wave (dispatch order): {start, end, HW_ID, XCC_ID}, or nullptr
#endif
};
// Several engines' fused T = 1 launches in ONE launch (fcx_run_group): member k's wave tiles
// are tiles [tile0, tile0 + af.n_tiles) of the grid.  Passed by value (kernel arguments).
constexpr int kMaxGroup = 4;
struct FinishGroup {
  int32_t n;
  int32_t nb[kMaxGroup];
  AtmosArgs a[kMaxGroup];
};
// cells per lane of the fp32 engine's fused kernels (16-B lanes of 4 floats; A/B builds: 2,
// 8-B lanes of 2 floats in 128-cell tiles like the fp64 kernels, half the registers per lane)
#ifndef FCX_F32_CPL
#define FCX_F32_CPL 4
#endif
constexpr int kF32Cpl = FCX_F32_CPL;
struct GroupMember {
  const Params *P;        // the member's device parameter block
  const double *corr_m;   // its month slice, or nullptr
  int64_t tile0;          // its first tile in the group's grid
  int32_t var;            // 1 CCLM, 2 MOM5, 3 RCO (the T = 1 specialisation)
  int32_t pad;
  AtmosFused af;          // its accumulation (af.n_tiles: its tile count)
};
// The grid's tiles in ranges: grid tiles [t0, next range's t0) are tiles [first, ...) of member
// `member`; a group launch has one range per member (all its tiles).  (Round 5 also launched
// the boundary-slot tiles apart, as ranges of the same members, to overlap the exchange; it
// measured slower and was removed in round 6.)
constexpr int kMaxGroupRanges = kMaxGroup;
struct GroupRange {
  int64_t t0;
  int64_t first;
  int32_t member;
  int32_t pad;
};
struct GroupArgs {
  int32_t n;
  int32_t n_ranges;
  int64_t total_tiles;
  GroupMember m[kMaxGroup];
  GroupRange r[kMaxGroupRanges];
};
// lc: the members' common launch shape (nontemporal, f32, halo > 0 or not); af.n_tiles of
// every member is set by the caller.  hipError_t as int.
int launch_cells_group(GroupMember *members, int n, const LaunchConfig &lc, void *stream);

// the segments carried over a tile boundary: carry of tile t-1 + the head cells of tile t,
// for every tile of a launch of n_cells (fp32: 256-cell tiles of float fields)
int launch_atmos_fixup(const AtmosFused &af, int64_t n_cells, bool f32, void *stream);
// zero the fused outputs of the n atmosphere cells in cells[] (cells without exchange cells)
int launch_atmos_zero(const AtmosFused &af, const int32_t *cells, int64_t n, bool f32, void *stream);
// the fix-ups of several engines' fused launches (fcx_run_group members) as one launch
struct FixupGroup {
  int32_t n;
  int32_t pad;
  int64_t first[kMaxGroup + 1];  // member m's (tile boundary, field) threads: [first[m], first[m+1])
  AtmosFused af[kMaxGroup];
};
int launch_atmos_fixup_group(const AtmosFused *afs, const int64_t *n_cells, int n, bool f32, void *stream);
int launch_atmos_finish(const AtmosArgs &a, int32_t n_boundaries, void *stream);

// f32: w, src and dst are float arrays (the reference's single-precision build, where the
// matrix weights and the fields are REAL(wp) = REAL(4), basic:117-122, and so is the sum)
// src and dst: engine buffers in the layout tpad
int launch_regrid_csr(const int32_t *row_ptr, const int32_t *col, const double *w,
                      const double *src, double *dst, int64_t n_dst, void *stream, bool f32 = false,
                      int64_t tpad = 0);
int launch_zero(double *x, int64_t n, void *stream);

}  // namespace fcx
