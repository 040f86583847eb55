// fcx_kernels.hip -- CDNA4 (gfx950) kernels of the exchange-grid flux engine.
//
// cells_kernel: ONE fused pass over the exchange-grid cells for every flux of a coupling
// step (flux_calculator.F90:902-991): RBBR, QSUR(t,u,v), MEVA(+bias), HLAT, HSEN, UMOM,
// VMOM, RSDR and the type-0 averages.  The reference makes one pass over memory per flux
// and per surface type (7+ passes, one scalar call per cell); here every input array is
// read once and every output written once, so the kernel is HBM-bandwidth bound
// (arithmetic intensity ~1.5-2 flop/B, well below the fp64-vector/HBM ridge).
//
// Layout: struct-of-arrays, one contiguous fp64 array per (surface type, grid, var) --
// exactly the reference data model (flux_calculator_basic.F90:86-103), so a wave reads
// 64 x 16 B = 1 KiB per array per load instruction (two cells per lane, dwordx4).
// Method dispatch (namelist which_* strings, calc:37-48 etc.) is a per-type int8 read
// from the parameter block: wave-uniform, so it is a scalar branch and costs no
// divergence.  Surface types are processed type-major per cell; every cross-type effect
// the reference's flux-major order has (the 'copy' aliases, the bias added once more per
// aliased copy, calc:112-116) is resolved by the planner in fcx_engine.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include "fcx_internal.h"
#include "fcx_physics.h"

#pragma clang fp contract(off)

namespace fcx {

// C cells of one lane in the arithmetic type R.  The fp64 path holds 2 cells per lane and
// the fp32 path 4, so one lane's access to an array is a single 16-B dwordx4 either way.
template <int C, class R = double>
struct Vec {
  R v[C];
};

typedef double d2 __attribute__((ext_vector_type(2)));
#if FCX_WAVE_TRACE
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
#endif
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef int i2v __attribute__((ext_vector_type(2)));
typedef int i4v __attribute__((ext_vector_type(4)));

// Field, map and output pointers reach the kernels through the parameter block as generic
// pointers, which the compiler lowers to FLAT loads and stores.  A FLAT access counts in
// both vmcnt and lgkmcnt, so every s_waitcnt lgkmcnt(0) that waits for a scalar load (the
// next array pointer out of the parameter block) also waits for all of the wave's loads in
// flight.  These are device (or host-mapped) arrays, never LDS or scratch: addressing them
// in the global address space gives GLOBAL instructions, counted in vmcnt alone.
// (Round 3: step -0.4 % fp64, -0.7 % fp32, -1.0 % at T = 2 against FLAT, profiles/r03/global_as_ab/.)
#define FCX_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ const FCX_GLOBAL T *gptr(const T *p) {
  return (const FCX_GLOBAL T *)p;
}
template <class T>
__device__ __forceinline__ FCX_GLOBAL T *gptr(T *p) {
  return (FCX_GLOBAL T *)p;
}

// NT: streamed once -> non-temporal hint (the arrays are read once and written once per
// step; the 256 MB Infinity Cache cannot hold a 10M-cell step anyway).  Out-of-range lanes
// of a partial vector read 1 (keeps exp/pow/division of the dead lanes finite).
template <int C, bool NT, class R>
__device__ __forceinline__ Vec<C, R> ld(const R *__restrict__ p, int64_t j0, int64_t n) {
  Vec<C, R> r;
  if constexpr (C * sizeof(R) == 16 || (C == 2 && sizeof(R) == 4)) {
    if (j0 + C <= n) {
      using V = typename std::conditional<sizeof(R) == 8, d2, typename std::conditional<C == 4, f4, f2v>::type>::type;
      const FCX_GLOBAL V *q = gptr(reinterpret_cast<const V *>(p + j0));
      const V t = NT ? __builtin_nontemporal_load(q) : *q;
#pragma unroll
      for (int i = 0; i < C; ++i) r.v[i] = t[i];
      return r;
    }
  }
#pragma unroll
  for (int i = 0; i < C; ++i) r.v[i] = (j0 + i < n) ? gptr(p)[j0 + i] : R(1);
  return r;
}

template <int C, bool NT, class R>
__device__ __forceinline__ void st(R *__restrict__ p, int64_t j0, int64_t n, const Vec<C, R> &x) {
  if constexpr (C * sizeof(R) == 16 || (C == 2 && sizeof(R) == 4)) {
    if (j0 + C <= n) {
      using V = typename std::conditional<sizeof(R) == 8, d2, typename std::conditional<C == 4, f4, f2v>::type>::type;
      FCX_GLOBAL V *q = gptr(reinterpret_cast<V *>(p + j0));
      V t;
#pragma unroll
      for (int i = 0; i < C; ++i) t[i] = x.v[i];
      // (write-through sc1 / sc1 nt stores instead of nt: step +9 to +27 %,
      // profiles/r03/store_wt_ab/ -- the L2 write-back merges the output lines)
      if (NT)
        __builtin_nontemporal_store(t, q);
      else
        *q = t;
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < C; ++i)
    if (j0 + i < n) gptr(p)[j0 + i] = x.v[i];
}

template <int C, class R>
__device__ __forceinline__ Vec<C, R> splat(R a) {
  Vec<C, R> r;
#pragma unroll
  for (int i = 0; i < C; ++i) r.v[i] = a;
  return r;
}

// The parameter block holds every field pointer as double*; in the fp32 engine the same
// pointers address float arrays, so every access reinterprets them as R*.
#define FOR_C _Pragma("unroll") for (int i = 0; i < C; ++i)
// Field arrays may be tile-blocked (fcx_internal.h, FCX_OPT_TILED_LAYOUT): cell j is at
// p + j + D_ with D_ = (j >> kLayoutShift) * tpad, the same shift for every array and for
// the C cells of one lane (j0 is a multiple of C, C divides the tile).  D_ is in scope
// wherever these are used; D_ = 0 for contiguous arrays.
#define LD(p, j, n) ld<C, NT, R>(reinterpret_cast<const R *>(p) + D_, j, n)
#define ST(p, j, n, ...) st<C, NT, R>(reinterpret_cast<R *>(p) + D_, j, n, __VA_ARGS__)

// Momentum of one (type, u- or v-grid) cell group; `north` selects VMOM.
struct NoEmit {
  template <int C, class R>
  __device__ __forceinline__ void operator()(int, const Vec<C, R> &) const {}
};

template <int C, bool NT, class R, class Emit>
__device__ __forceinline__ void momentum(int8_t m, bool north, const UVGridPtrs &g,
                                         const Vec<C, R> &ts, const Vec<C, R> &ps, const Vec<C, R> &u,
                                         const Vec<C, R> &v, const Vec<C, R> &vel, const Vec<C, R> &qs,
                                         const Vec<C, R> &a, int64_t j0, int64_t n, int64_t D_, Emit &emit, int slot);

template <int C, bool NT, class R>
__device__ __forceinline__ void momentum(int8_t m, bool north, const UVGridPtrs &g,
                                         const Vec<C, R> &ts, const Vec<C, R> &ps, const Vec<C, R> &u,
                                         const Vec<C, R> &v, const Vec<C, R> &vel, const Vec<C, R> &qs,
                                         const Vec<C, R> &a, int64_t j0, int64_t n, int64_t D_) {
  NoEmit none;
  momentum<C, NT, R>(m, north, g, ts, ps, u, v, vel, qs, a, j0, n, D_, none, -1);
}

template <int C, bool NT, class R, class Emit>
__device__ __forceinline__ void momentum(int8_t m, bool north, const UVGridPtrs &g,
                                         const Vec<C, R> &ts, const Vec<C, R> &ps, const Vec<C, R> &u,
                                         const Vec<C, R> &v, const Vec<C, R> &vel, const Vec<C, R> &qs,
                                         const Vec<C, R> &a, int64_t j0, int64_t n, int64_t D_, Emit &emit, int slot) {
  if (!g.mom) return;
  Vec<C, R> out;
  if (m == FCX_ZERO) {
    out = splat<C, R>(R(0));
  } else if (m == FCX_CCLM || m == FCX_MOM5) {
    FOR_C {
      const R rate = mom_cclm_rate(a.v[i], ps.v[i], qs.v[i], ts.v[i], vel.v[i]);
      out.v[i] = -(rate * (north ? v.v[i] : u.v[i]));
    }
  } else if (m == FCX_RCO) {
    FOR_C {
      const R rate = mom_rco_rate(vel.v[i]);
      out.v[i] = -(rate * (north ? v.v[i] : u.v[i]));
    }
  } else {
    return;
  }
  ST(g.mom, j0, n, out);
  if (slot >= 0) emit(slot, out);
}

// QSUR + momentum on one separate u or v grid (non-merged layout).
template <int C, bool NT, class R>
__device__ __forceinline__ void uv_grid(const TypeParams &tp, int k, uint32_t stages, int64_t j0,
                                        int64_t n, int64_t D_) {
  const UVGridPtrs &g = tp.uv[k];
  const uint32_t s_qsur = k == 0 ? S_QSUR_U : S_QSUR_V;
  const uint32_t s_mom = k == 0 ? S_UMOM : S_VMOM;
  const bool do_q = (stages & s_qsur) && tp.m_qsur[1 + k] == FCX_CCLM && g.qsur;
  const bool do_m = (stages & s_mom) && g.mom;
  if (!do_q && !do_m) return;
  Vec<C, R> ts = {}, fi = {}, ps = {}, u = {}, v = {}, a = {}, qs = {};
  if (g.tsur) ts = LD(g.tsur, j0, n);
  if (g.psur) ps = LD(g.psur, j0, n);
  // every load is guarded by its own pointer, whatever the method says: a method whose input
  // the planner left unbound reads nothing (plan_audit at plan build names that case as an
  // error before any launch; round-5 fault: 'zero' momentum loaded unbound winds)
  if (do_q && g.fice) fi = LD(g.fice, j0, n);
  if (do_m) {  // ('zero' momentum binds no wind: the planner leaves uatm / vatm unset)
    if (g.uatm) u = LD(g.uatm, j0, n);
    if (g.vatm) v = LD(g.vatm, j0, n);
    if (tp.m_mom == FCX_CCLM && g.amom) a = LD(g.amom, j0, n);
    if (tp.m_mom == FCX_MOM5 && g.cmom) a = LD(g.cmom, j0, n);
    if (g.qsur_in && !do_q) qs = LD(g.qsur_in, j0, n);
  }
  if (do_q) {
    FOR_C qs.v[i] = qsur_cclm(fi.v[i], ps.v[i], ts.v[i]);
    ST(g.qsur, j0, n, qs);
  }
  if (do_m) {
    Vec<C, R> vel;
    FOR_C vel.v[i] = wind(u.v[i], v.v[i]);
    momentum<C, NT, R>(tp.m_mom, k == 1, g, ts, ps, u, v, vel, qs, a, j0, n, D_);
  }
}

// LDS accumulators of the register-average slots: each lane owns C contiguous values per
// slot (16 B), slot k at base + k * stride.  Private to the lane, so no synchronisation;
// they keep 7 x C values out of the VGPR budget of the multi-type kernels.
template <int C, class R>
struct AccLds {
  R *base;
  int stride;  // elements between slots
  __device__ __forceinline__ Vec<C, R> get(int k) const {
    Vec<C, R> r;
#pragma unroll
    for (int i = 0; i < C; ++i) r.v[i] = base[k * stride + i];
    return r;
  }
  __device__ __forceinline__ void set(int k, const Vec<C, R> &x) const {
#pragma unroll
    for (int i = 0; i < C; ++i) base[k * stride + i] = x.v[i];
  }
};

// Where a produced flux goes besides its own array.  RAVG: X_s * FARE_s is added to the
// type-0 accumulator of its slot (type order, from 0.0 -- calc:377-383) and the averages
// go to the emitter (the fused atmosphere accumulation) once all types are done; without
// RAVG the value of the single surface type goes to the emitter.
template <int C, class R, bool RAVG, class Emit>
struct Sink {
  const Emit &emit;
  const AvgRegs &ra;
  AccLds<C, R> acc;
  Vec<C, R> fare;
  __device__ __forceinline__ Sink(const Emit &e, const AvgRegs &r, AccLds<C, R> a) : emit(e), ra(r), acc(a) {
    if constexpr (RAVG) {
#pragma unroll
      for (int k = 0; k < kAvgSlots; ++k)
        if (ra.out[k]) acc.set(k, splat<C, R>(R(0)));
    }
  }
  __device__ __forceinline__ void operator()(int k, const Vec<C, R> &x) {
    if constexpr (RAVG) {
      if (ra.out[k]) {
        Vec<C, R> a = acc.get(k);
#pragma unroll
        for (int i = 0; i < C; ++i) a.v[i] = a.v[i] + x.v[i] * fare.v[i];
        acc.set(k, a);
      }
    } else {
      if (k < kFusedFields) emit(k, x);
    }
  }
};

// Remap records (Params::rec): every flux of register slot k the T=1 launch produces is also
// stored at position rec_pos[k] of its cell's record, so that a remap of those fields
// gathers one record per link without a packing pass (fcx_engine.hip plan_fused_records).
template <int C, class R, class Inner>
struct RecEmit {
  const Inner &inner;
  R *rec;             // record of the lane's first cell
  int P;              // elements per record
  const int8_t *pos;  // Params::rec_pos (wave-uniform)
  int nv;             // cells of the lane inside the grid
#ifndef FCX_REC_VEC  // 1: the values stay in registers and each record goes out as 16-B stores
#define FCX_REC_VEC 1
#endif
  mutable R vals[6][C];
  template <int CC, class RR>
  __device__ __forceinline__ void operator()(int k, const Vec<CC, RR> &x) const {
    inner(k, x);
    if (FCX_REC_VEC) {
      if (k < 6) {
#pragma unroll
        for (int i = 0; i < CC; ++i) vals[k][i] = x.v[i];
      }
      return;
    }
    const int p = pos[k];
    if (p >= 0) {
#pragma unroll
      for (int i = 0; i < CC; ++i)
        if (i < nv) gptr(rec)[i * P + p] = x.v[i];
    }
  }
  __device__ __forceinline__ void flush() const {
    if (!FCX_REC_VEC) return;
    constexpr int V = 16 / sizeof(R);
#pragma unroll
    for (int i = 0; i < C; ++i) {
      if (i >= nv) break;
#pragma unroll
      for (int q = 0; q < 6 / V; ++q) {
        if (q * V >= P) break;
        using VecT = typename std::conditional<sizeof(R) == 8, d2, f4>::type;
        VecT t;
#pragma unroll
        for (int h = 0; h < V; ++h) {
          R v = R(0);
#pragma unroll
          for (int k = 0; k < 6; ++k)
            if (pos[k] == q * V + h) v = vals[k][i];
          t[h] = v;
        }
        *gptr(reinterpret_cast<VecT *>(rec + i * P + q * V)) = t;
      }
    }
  }
};

// VAR: 0 = generic (methods read from the parameter block); 1/2/3 = the CCLM / MOM5 / RCO
// variant with the QSUR/MEVA/HSEN/momentum methods of every surface type fixed at compile
// time, so the other method paths vanish from the code and its register budget.  Any T.
// Inputs shared by consecutive surface types (the atmosphere fields are aliased into every
// type, basic:334-358) are loaded once: a type reloads an input only when its pointer
// differs from the previous type's (wave-uniform scalar compare).  Inputs are never written
// by the pass, so a held value is the array's value.
// TM: 1 = one surface type, fixed at compile time (the held inputs and the type loop
// vanish); 0 = T from the parameter block.  RAVG (register averages) needs TM = 0.
// HALO: cells at or past st_end are a halo tile's head cells -- their fluxes are computed for
// the fused accumulation's products, nothing of them is stored (the next tile's wave stores).
template <int C, bool MERGED, int VAR, bool NT, class R = double, int TM = 1, bool RAVG = false,
          class Emit = NoEmit, bool REC = false, bool HALO = false>
__device__ __forceinline__ void process(const Params *__restrict__ P, const double *__restrict__ corr_m,
                                        int64_t j0, const Emit &emit_in = Emit(),
                                        AccLds<C, R> acc_lds = AccLds<C, R>{nullptr, 0}, int64_t st_end = 0) {
  static_assert(!(RAVG && TM), "register averages need more than one surface type");
  static_assert(!REC || (TM == 1 && !RAVG), "remap records: the T=1 launch");
  static_assert(!HALO || (TM == 1 && !RAVG) || (FCX_HALO_RAVG && RAVG), "halo tiles: the T=1 launch");
  const uint32_t stages = P->stages;
  const int T = TM ? 1 : P->num_types;
  const int64_t nt = P->n[0];
  const int64_t ns = HALO ? min(nt, st_end) : nt;  // stores of the t-grid (and merged u/v) cells
  const bool do_t = j0 < nt;
  using SinkEmit = typename std::conditional<REC, RecEmit<C, R, Emit>, const Emit &>::type;
  SinkEmit emit = [&]() -> SinkEmit {
    if constexpr (REC)
      return RecEmit<C, R, Emit>{emit_in, reinterpret_cast<R *>(P->rec) + j0 * P->rec_p, P->rec_p, P->rec_pos,
                                 (int)max((int64_t)0, min((int64_t)C, ns - j0))};
    else
      return emit_in;
  }();
  const int64_t D_ = (j0 >> kLayoutShift) * P->tpad;  // field layout shift of this lane's cells
  Vec<C, R> corr = {};  // the month slice is a plain contiguous array
  if (do_t && corr_m && (stages & S_MEVA)) corr = ld<C, NT, R>(reinterpret_cast<const R *>(corr_m), j0, nt);
  Vec<C, R> rsdd = {};
  if (do_t && P->rsdd0 && (stages & S_RSDR)) rsdd = LD(P->rsdd0, j0, nt);
  Sink<C, R, RAVG, typename std::remove_cv<typename std::remove_reference<SinkEmit>::type>::type> sink(
      emit, P->ravg, acc_lds);

  // inputs held across surface types, with the pointer they were loaded from
  Vec<C, R> ts = {}, fi = {}, ps = {}, pa = {}, qa = {}, ta = {}, u = {}, v = {}, amoi = {}, cmoi = {},
            chea = {}, amom = {}, cmom = {}, vel = {};
  const double *h_ts = nullptr, *h_fi = nullptr, *h_ps = nullptr, *h_pa = nullptr, *h_qa = nullptr,
               *h_ta = nullptr, *h_u = nullptr, *h_v = nullptr, *h_amoi = nullptr, *h_cmoi = nullptr,
               *h_chea = nullptr, *h_amom = nullptr, *h_cmom = nullptr;
  // With T from the parameter block (TM = 0) the bottom-side inputs (TSUR FICE CMOI CHEA
  // CMOM) are reloaded for every type, and the atmosphere-side inputs (PSUR PATM QATM TATM
  // UATM VATM AMOI AMOM, aliased into every surface type by distribute_input_field,
  // basic:334-358) are held across the types and reloaded only when a type binds another
  // array (a wave-uniform pointer compare).  Measured at T = 2 (profiles/r02/t2_reload_ab):
  // the per-type reloads of the shared fields cost 8 % of the step; holding them costs 36
  // VGPRs, so the multi-type fused kernels run 3 instead of 4 waves per SIMD and still gain
  // 6-7 % per step.  Holding every input (round 1) kept ~56 VGPRs live and lost.
  constexpr bool kReload = TM == 0;  // bottom-side inputs: loaded per type
  // grp.member names the pointer in TypeParams.  ATM: an atmosphere-side input (held).
#define HOLDX(var, grp, member, ATM)                  \
  {                                                   \
    const double *ptr_ = tp.grp.member;               \
    if constexpr (kReload && !ATM) {                  \
      if (ptr_) var = LD(ptr_, j0, nt);               \
    } else if (ptr_ && ptr_ != h_##var) {             \
      var = LD(ptr_, j0, nt);                         \
      h_##var = ptr_;                                 \
    }                                                 \
  }
#define HOLD(var, grp, member) HOLDX(var, grp, member, false)
#define HOLDA(var, grp, member) HOLDX(var, grp, member, true)
  // Next-type prefetch (multi-type kernels): the bottom-side inputs of type s+1 (TSUR FICE
  // CMOI CHEA CMOM and the FARE of the averages) are loaded when type s starts, so that the
  // wave does not stall on memory between two types.  The fused T = 2 kernels then hold
  // 162 / 166 / 124 VGPRs (CCLM / MOM5 / RCO, was 150 / 144 / 116): still 3 / 3 / 4 waves per
  // SIMD, no spills.  In one process over the same arrays (profiles/r03/ab_t2_prefetch.json,
  // random map): T = 2 step 1.672 -> 1.625 ms, CCLM 5.14 -> 5.26 TB/s, MOM5 5.54 -> 5.67,
  // RCO 5.26 -> 5.50.
#ifndef FCX_T2_PREFETCH  // A/B builds: 0 = no next-type prefetch (24 fewer VGPRs)
#define FCX_T2_PREFETCH 1
#endif
  constexpr bool kPrefetch = kReload && FCX_T2_PREFETCH;
  // Multi-type CCLM / MOM5 kernels: the atmosphere-only terms of the formulas are formed once
  // per cell, when the type's atmosphere fields are (re)loaded, instead of once per type:
  // T_a * EF (HSEN's pow, ta_exner) and, for CCLM, whose coefficients AMOI / AMOM are
  // atmosphere fields too, a * max(vel, u_min) * p_s (MEVA, HSEN) and a * vel * p_s
  // (momentum).  Same operations on the same values, so the same bits (fcx_physics.h); the
  // type loop loses its pow and PATM / AMOI / AMOM / the wind speed need not stay live.
  // (round 4, in one process over the same arrays, profiles/r04/ab/ab_derive_t2.json: T = 2 step
  // 1.665 -> 1.628 ms, MOM5 0.616 -> 0.582 ms, CCLM 0.595 -> 0.588 ms)
  constexpr bool kDerive = TM == 0 && (VAR == 1 || VAR == 2);
  Vec<C, R> taef = {}, amv = {}, mvp = {};
  Vec<C, R> n_ts = {}, n_fi = {}, n_cmoi = {}, n_chea = {}, n_cmom = {}, n_fare = {};
  auto prefetch = [&](int s2) {
    const TypeParams &q = P->type[s2];
    if (q.t.tsur) n_ts = LD(q.t.tsur, j0, nt);
    if (q.t.fice) n_fi = LD(q.t.fice, j0, nt);
    if (q.t.cmoi) n_cmoi = LD(q.t.cmoi, j0, nt);
    if (q.t.chea) n_chea = LD(q.t.chea, j0, nt);
    if constexpr (MERGED) {
      if (q.uv[0].cmom) n_cmom = LD(q.uv[0].cmom, j0, nt);
    }
    if constexpr (RAVG) {
      if (P->ravg_on && P->ravg.fare[s2]) n_fare = LD(P->ravg.fare[s2], j0, nt);
    }
  };
  if constexpr (kPrefetch) {
    if (do_t) prefetch(0);
  }

  for (int s = 0; s < T; ++s) {
    if constexpr (kReload) {  // no bottom-side input of the previous type stays live
      ts = fi = cmoi = chea = cmom = Vec<C, R>{};
    }
    const TypeParams &tp = P->type[s];
    const TGridPtrs &g = tp.t;
    constexpr int8_t kVarMethod = VAR == 1 ? FCX_CCLM : VAR == 2 ? FCX_MOM5 : FCX_RCO;
    const int8_t m_q = VAR ? (VAR == 3 ? FCX_NONE : FCX_CCLM) : tp.m_qsur[0];
    const int8_t m_qu = VAR ? m_q : tp.m_qsur[1];
    const int8_t m_qv = VAR ? m_q : tp.m_qsur[2];
    const int8_t m_me = VAR ? kVarMethod : tp.m_meva;
    const int8_t m_hs = VAR ? kVarMethod : tp.m_hsen;
    const int8_t m_mo = VAR ? kVarMethod : tp.m_mom;
    if (do_t) {
      // ---- every t-grid input this type needs (before any store of this type)
      Vec<C, R> qs = {}, me = {};
      if constexpr (kPrefetch) {
        ts = n_ts;
        fi = n_fi;
        cmoi = n_cmoi;
        chea = n_chea;
        cmom = n_cmom;
        if constexpr (RAVG) sink.fare = n_fare;
        if (s + 1 < T) prefetch(s + 1);
      } else {
        HOLD(ts, t, tsur)
        HOLD(fi, t, fice)
      }
      // which derived atmosphere terms this type must (re)form: its fields differ from the held ones
      const bool wind_new = (g.uatm && g.uatm != h_u) || (g.vatm && g.vatm != h_v);
      bool d_ef = false, d_amv = false, d_mvp = false;
      if constexpr (kDerive) {
        const bool ps_new = g.psur && g.psur != h_ps;
        d_ef = ps_new || (g.patm && g.patm != h_pa) || (g.tatm && g.tatm != h_ta);
        if constexpr (VAR == 1) {
          d_amv = ps_new || wind_new || (g.amoi && g.amoi != h_amoi);
          d_mvp = ps_new || wind_new || (tp.uv[0].amom && tp.uv[0].amom != h_amom);
        }
      }
      HOLDA(ps, t, psur)
      if constexpr (!kDerive) HOLDA(pa, t, patm)
      HOLDA(qa, t, qatm)
      HOLDA(ta, t, tatm)
      HOLDA(u, t, uatm)
      HOLDA(v, t, vatm)
      if constexpr (!(kDerive && VAR == 1)) HOLDA(amoi, t, amoi)
      if constexpr (kDerive) {
        if (d_ef) {
          Vec<C, R> pa_l = {};
          if (g.patm) pa_l = LD(g.patm, j0, nt);
          h_pa = g.patm;
          FOR_C taef.v[i] = ta_exner(ta.v[i], ps.v[i], pa_l.v[i]);
        }
        if constexpr (VAR == 1) {
          if (d_amv || d_mvp) {
            Vec<C, R> w;  // the wind speed, only to form the two factors
            FOR_C w.v[i] = wind(u.v[i], v.v[i]);
            if (d_amv) {
              Vec<C, R> am = {};
              if (g.amoi) am = LD(g.amoi, j0, nt);
              h_amoi = g.amoi;
              FOR_C amv.v[i] = rate_num(am.v[i], w.v[i], ps.v[i]);
            }
            if (d_mvp) {
              Vec<C, R> am = {};
              if (tp.uv[0].amom) am = LD(tp.uv[0].amom, j0, nt);
              h_amom = tp.uv[0].amom;
              FOR_C mvp.v[i] = mom_num(am.v[i], w.v[i], ps.v[i]);
            }
          }
        }
      }
      if constexpr (!kPrefetch) {
        HOLD(cmoi, t, cmoi)
        HOLD(chea, t, chea)
      }
      if (g.qsur_in) qs = LD(g.qsur_in, j0, nt);  // may be written by this pass: never held
      if (g.meva_in) me = LD(g.meva_in, j0, nt);
      if constexpr (MERGED) {
        if constexpr (!(kDerive && VAR == 1)) HOLDA(amom, uv[0], amom)
        if constexpr (!kPrefetch) HOLD(cmom, uv[0], cmom)
      }
      if constexpr (!(kDerive && VAR == 1)) {
        if (wind_new) FOR_C vel.v[i] = wind(u.v[i], v.v[i]);
      }
      if constexpr (RAVG) {
        if constexpr (!kPrefetch) {
          if (P->ravg_on && P->ravg.fare[s]) sink.fare = LD(P->ravg.fare[s], j0, nt);
        }
        sink(A_TSUR, ts);
      }


      // ---- calc_flux_radiation_blackbody (calc:331-343)
      if ((stages & S_RBBR) && g.rbbr) {
        Vec<C, R> r;
        if (tp.m_rbbr == FCX_STBO) {
          FOR_C r.v[i] = rbbr_stbo(ts.v[i]);
          ST(g.rbbr, j0, ns, r);
          sink(A_RBBR, r);
        } else if (tp.m_rbbr == FCX_ZERO) {
          ST(g.rbbr, j0, ns, splat<C, R>(R(0)));
          sink(A_RBBR, splat<C, R>(R(0)));
        }
      }
      // ---- calc_spec_vapor_surface(t) (calc:37-49)
      if ((stages & S_QSUR_T) && m_q == FCX_CCLM) {
        FOR_C qs.v[i] = qsur_cclm(fi.v[i], ps.v[i], ts.v[i]);
        if (g.qsur) ST(g.qsur, j0, ns, qs);
      }
      // ---- calc_flux_mass_evap (calc:75-118), P2: TATM in the T_s slot
      if (stages & S_MEVA) {
        const int8_t m = m_me;
        bool have = true;
        if (m == FCX_ZERO) {
          me = splat<C, R>(R(0));
        } else if (m == FCX_CCLM || m == FCX_MOM5) {
          if constexpr (kDerive && VAR == 1) {
            FOR_C me.v[i] = meva_cclm_num(amv.v[i], qa.v[i], qs.v[i], ta.v[i]);
          } else {
            const Vec<C, R> &a = (m == FCX_CCLM) ? amoi : cmoi;
            FOR_C me.v[i] = meva_cclm(a.v[i], ps.v[i], qa.v[i], qs.v[i], ta.v[i], vel.v[i]);
          }
        } else if (m == FCX_RCO) {
          FOR_C me.v[i] = meva_rco(qa.v[i], ts.v[i], vel.v[i]);
        } else {
          have = false;  // none / copy
        }
        if (have) {
          for (int b = 0; b < tp.bias_adds; ++b) {
            FOR_C me.v[i] = me.v[i] + corr.v[i];
          }
          if (g.meva) ST(g.meva, j0, ns, me);
          sink(A_MEVA, me);
        }
      }
      // ---- calc_flux_heat_latent (calc:135-152)
      if ((stages & S_HLAT) && g.hlat) {
        Vec<C, R> h;
        if (tp.m_hlat == FCX_WATER) {
          FOR_C h.v[i] = me.v[i] * R(kLv);
          ST(g.hlat, j0, ns, h);
        } else if (tp.m_hlat == FCX_ICE) {
          FOR_C h.v[i] = me.v[i] * R(kLs);
          ST(g.hlat, j0, ns, h);
        } else if (tp.m_hlat == FCX_ZERO) {
          h = splat<C, R>(R(0));
          ST(g.hlat, j0, ns, h);
        }
        if (tp.m_hlat == FCX_WATER || tp.m_hlat == FCX_ICE || tp.m_hlat == FCX_ZERO) sink(A_HLAT, h);
      }
      // ---- calc_flux_heat_sensible (calc:167-206), P3: QATM in the q_s slot
      if ((stages & S_HSEN) && g.hsen) {
        const int8_t m = m_hs;
        Vec<C, R> h;
        if (m == FCX_CCLM || m == FCX_MOM5) {
          if constexpr (kDerive && VAR == 1) {
            FOR_C h.v[i] = hsen_cclm_num(amv.v[i], qa.v[i], ts.v[i], taef.v[i]);
          } else if constexpr (kDerive) {
            FOR_C h.v[i] = hsen_cclm_num(rate_num(chea.v[i], vel.v[i], ps.v[i]), qa.v[i], ts.v[i], taef.v[i]);
          } else {
            const Vec<C, R> &a = (m == FCX_CCLM) ? amoi : chea;
            FOR_C h.v[i] = hsen_cclm(a.v[i], pa.v[i], ps.v[i], qa.v[i], ta.v[i], ts.v[i], vel.v[i]);
          }
          ST(g.hsen, j0, ns, h);
        } else if (m == FCX_RCO) {
          FOR_C h.v[i] = hsen_rco(ta.v[i], ts.v[i], vel.v[i]);
          ST(g.hsen, j0, ns, h);
        } else if (m == FCX_ZERO) {
          h = splat<C, R>(R(0));
          ST(g.hsen, j0, ns, h);
        }
        if (m == FCX_CCLM || m == FCX_MOM5 || m == FCX_RCO || m == FCX_ZERO) sink(A_HSEN, h);
      }
      if constexpr (MERGED) {
        // u and v grids ARE the t grid: QSUR(u/v) = QSUR(t) (same inputs, same method),
        // one wind speed and one exchange rate serve UMOM and VMOM.
        for (int k = 0; k < 2; ++k) {
          const UVGridPtrs &gk = tp.uv[k];
          const uint32_t s_qsur = k == 0 ? S_QSUR_U : S_QSUR_V;
          if ((stages & s_qsur) && (k == 0 ? m_qu : m_qv) == FCX_CCLM && gk.qsur) {
            if (!((stages & S_QSUR_T) && m_q == FCX_CCLM)) {
              FOR_C qs.v[i] = qsur_cclm(fi.v[i], ps.v[i], ts.v[i]);
            }
            ST(gk.qsur, j0, ns, qs);
          }
        }
        const bool do_u = (stages & S_UMOM) && tp.uv[0].mom;
        const bool do_v = (stages & S_VMOM) && tp.uv[1].mom;
        if (do_u || do_v) {
          if constexpr (kDerive && VAR == 1) {  // CCLM: the rate from a * vel * p_s formed once
            Vec<C, R> rate;
            FOR_C rate.v[i] = mom_cclm_rate_num(mvp.v[i], qs.v[i], ts.v[i]);
            for (int k = 0; k < 2; ++k) {
              if (!(k ? do_v : do_u)) continue;
              Vec<C, R> out;
              FOR_C out.v[i] = -(rate.v[i] * (k ? v.v[i] : u.v[i]));
              ST(tp.uv[k].mom, j0, ns, out);
              sink(k ? A_VMOM : A_UMOM, out);
            }
          } else {
            const Vec<C, R> &a = (m_mo == FCX_MOM5) ? cmom : amom;
            if (do_u) momentum<C, NT, R>(m_mo, false, tp.uv[0], ts, ps, u, v, vel, qs, a, j0, ns, D_, sink, A_UMOM);
            if (do_v) momentum<C, NT, R>(m_mo, true, tp.uv[1], ts, ps, u, v, vel, qs, a, j0, ns, D_, sink, A_VMOM);
          }
        }
      }
      // ---- distribute_shortwave_radiation_flux (calc:355-362): RSDR_s = RSDD_0
      if ((stages & S_RSDR) && g.rsdr) ST(g.rsdr, j0, ns, rsdd);
    }
    if constexpr (!MERGED) {
      if (j0 < P->n[1]) uv_grid<C, NT, R>(tp, 0, stages, j0, P->n[1], D_);
      if (j0 < P->n[2]) uv_grid<C, NT, R>(tp, 1, stages, j0, P->n[2], D_);
    }
  }
#undef HOLD
#undef HOLDA
#undef HOLDX

  if constexpr (REC) emit.flush();
  // ---- average_across_surface_types (calc:376-383), summed in type order
  if constexpr (RAVG) {
    if (do_t) {
#pragma unroll
      for (int k = 0; k < kAvgSlots; ++k) {
        if (!P->ravg.out[k]) continue;
        const Vec<C, R> avg = sink.acc.get(k);
        ST(P->ravg.out[k], j0, ns, avg);
        if (k < kFusedFields) emit(k, avg);  // the type-0 field OASIS sends on
      }
    }
  }
  if (stages & S_AVG) {
    for (int e = 0; e < P->num_avg; ++e) {
      const AvgEntry &ae = P->avg[e];
      const int64_t n = P->n[ae.grid];
      if (j0 >= n) continue;
      Vec<C, R> acc = splat<C, R>(R(0));
      if (!ae.x0) continue;  // (plan_audit: every entry binds x0, x[s] and fare[s])
      for (int s = 0; s < T; ++s) {
        if (!ae.x[s] || !ae.fare[s]) continue;
        const Vec<C, R> x = LD(ae.x[s], j0, n);
        const Vec<C, R> f = LD(ae.fare[s], j0, n);
        FOR_C acc.v[i] = acc.v[i] + x.v[i] * f.v[i];
      }
      ST(ae.x0, j0, HALO ? min(n, st_end) : n, acc);
    }
  }
}

// cells [lo, hi) of the plan (lo a multiple of C), grid-stride over C-cell units
template <int C, bool MERGED, int VAR, bool NT, class R, int TM, bool RAVG, bool REC = false>
__global__ __launch_bounds__(256, RAVG ? 3 : 1) void cells_kernel(const Params *__restrict__ P,
                                                    const double *__restrict__ corr_m, int64_t lo,
                                                    int64_t hi) {
  const int64_t u_end = (hi + C - 1) / C;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // register-average accumulators: [slot][thread][C] (16 B per lane and slot, conflict-free)
  __shared__ R s_acc[RAVG ? kAvgSlots * 256 * C : 1];
  const AccLds<C, R> acc{s_acc + threadIdx.x * C, 256 * C};
  for (int64_t u = lo / C + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < u_end; u += stride)
    process<C, MERGED, VAR, NT, R, TM, RAVG, NoEmit, REC>(P, corr_m, u * C, NoEmit(), acc);
}

// The T=1 hot path with the exchange -> atmosphere accumulation fused in (AtmosFused).
// Wave-uniform loop over 128-cell wave tiles (lane l: cells 2l, 2l+1).  Each flux is
// turned into the product w*x the moment it is produced and parked in the wave's own LDS
// region (nothing extra stays live in registers).  Segment boundaries come from two wave
// ballots of "this cell's atmosphere cell differs from the previous one": the lane holding
// a segment's first cell finds the segment end with a count-trailing-zeros, so after a
// wave-local fence it sums the segment's products from LDS in link order with a known trip
// count (no index re-reads, no dependent loop exit).  A segment that runs past the wave
// tile leaves its prefix in carry[tile].
// LDS row of one field: the products of cell e sit at slot(e) = e + 2*(e/16), i.e. one
// 16-B pad slot after every 16 cells.  Unpadded, cells 16 apart share a bank pair of the
// 16-lane ds_read2_b64 groups and the segment-start lanes (3-5 cells apart) collide; the
// pad shifts every 16-cell block by 2 banks and keeps the pair (2l, 2l+1) 16-B aligned.
// The fp32 engine's fused kernel holds C = 4 cells per lane: 256-cell wave tiles, rows of
// row_len<4>() products (the products and sums stay fp64, as in atmos_kernel).
template <int C>
constexpr int tile_cells() { return 64 * C; }
template <int C>
constexpr int row_len() { return tile_cells<C>() + 2 * (tile_cells<C>() / 16); }
__device__ __forceinline__ int lds_slot(int e) { return e + 2 * (e >> 4); }

// fp32 fields (the fp32 engine): the wave's LDS holds the fluxes themselves, [kFusedFields]
// rows of tile_cells<C>() floats, and one row of weights (fp64, lds_slot layout) behind them;
// the segment sums form w * (double)x as they read them -- the same products in the same
// order, in 4 instead of 6 row-lengths of fp64 per wave (more waves per CU).
template <int C>
constexpr int xrows_doubles() { return kFusedFields * tile_cells<C>() / 2; }
// fp32 (C = 4, up to 4 segment starts per lane): the tile's segments are summed by ordinal --
// segment s of the tile by lane s % 64 in round s / 64 -- so that each round's atmosphere
// stores are ONE contiguous run of atmosphere cells per field.  Summed by the lane holding
// its first cell (the fp64 rule, at most one start per lane there) the rounds interleave:
// round 1 takes every lane's first segment, round 2 the second ones in between, and each
// 128-B output line is written piecewise by two store instructions.  The list of the tile's
// segments sits behind the weights row: per segment its first cell and length - 1 (one byte
// each: a tile has 256 cells) and its atmosphere cell, room for one segment per cell (6 B x
// 256 = 192 doubles).  16 waves per CU then hold 156 KiB of LDS.
#ifndef FCX_F32_SEG_ORDINAL
#define FCX_F32_SEG_ORDINAL 1
#endif
constexpr int kSegCap = 192;  // doubles of the list (tile_cells<4>() x (2 + 4) bytes)
template <class R, int C>
constexpr bool seg_ordinal() { return FCX_F32_SEG_ORDINAL && sizeof(R) == 4 && C == 4; }
template <class R, int C>
constexpr int wave_lds_doubles(int rows) {
  return sizeof(R) == 4 ? xrows_doubles<C>() + row_len<C>() + (seg_ordinal<R, C>() ? kSegCap : 0)
                        : rows * row_len<C>();
}

template <int C>
struct LdsEmitT {
  double *p;    // this wave's [kFusedFields][row_len<C>()] products (fp32: flux rows, weights)
  double w[C];  // the weights of the lane's cells
  int s;        // lds_slot(C * lane)
  template <int CC, class R>
  __device__ __forceinline__ void operator()(int k, const Vec<CC, R> &x) const {
    static_assert(CC == C, "one emitter per cell width");
    if (FCX_DBG_ATM_NOLDS) return;
    if constexpr (sizeof(R) == 4 && C == 4) {  // one 16-B store of the lane's four fluxes
      const int lane = threadIdx.x & 63;
      *reinterpret_cast<f4 *>(reinterpret_cast<float *>(p) + k * tile_cells<C>() + C * lane) =
          f4{x.v[0], x.v[1], x.v[2], x.v[3]};
      return;
    } else if constexpr (sizeof(R) == 4 && C == 2) {  // (kF32Cpl 2: one 8-B store)
      const int lane = threadIdx.x & 63;
      *reinterpret_cast<f2v *>(reinterpret_cast<float *>(p) + k * tile_cells<C>() + C * lane) = f2v{x.v[0], x.v[1]};
      return;
    }
#pragma unroll
    for (int h = 0; h < C / 2; ++h) {  // 16-B LDS stores, w * x in fp64
      const d2 q = {w[2 * h] * (double)x.v[2 * h], w[2 * h + 1] * (double)x.v[2 * h + 1]};
      *reinterpret_cast<d2 *>(p + k * row_len<C>() + s + 2 * h) = q;
    }
  }
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lowest set bit index of m, 64 if none
__device__ __forceinline__ int first_bit(uint64_t m) { return m ? __builtin_ctzll(m) : 64; }

// XCD-aware block order.  Workgroups are dispatched round-robin over the 8 XCDs (block b on
// XCD b % 8), each XCD with its own L2.  Neighbouring tiles share the 128-B lines of the
// atmosphere outputs their segments end in; mapped to the same XCD, the two partial lines
// merge in that L2 before write-back instead of reaching memory as two partial writes.
// XCD runs (round 3): XCD x takes runs of FCX_XCD_CHUNK = 64 consecutive workgroups (256
// tiles), the 8 XCDs' runs side by side, so that only one tile edge in 256 is shared between
// two XCDs AND the chip streams from one window of the arrays, as the dispatch order
// advances.  Rounds 1-2 gave each XCD one contiguous eighth of the grid, b -> x * (nb / 8) +
// min(x, nb % 8) + b / 8: eight windows 1/8 of the arrays apart.  In one process over the
// same arrays, runs against eighths (profiles/r03/xcd_map_ab/): step -2.4 / -6.1 % fp64 (two
// boxes), -2.7 / -2.2 % fp32, -3.1 / -0.8 % at T = 2, -5.4 % on the periodic map.
constexpr uint32_t kXcds = 8;
#ifndef FCX_XCD_CHUNK  // workgroups per XCD run (fp64 kernels, 128-cell tiles)
#define FCX_XCD_CHUNK 64
#endif
#ifndef FCX_XCD_CHUNK_F32  // ... and of the fp32 kernels (256-cell tiles): 16 against 64,
#define FCX_XCD_CHUNK_F32 32  // step -0.7 % (shared arrays) / -4.0 % (own mirrors),
#endif                        // profiles/r03/xcd_map_ab/f32_*; round 5, the fp32 group launch:
                              // 32 against 16 -1.0 / -1.2 % (two boxes), 64 -0.2 %, and with
                              // the ordinal segment rounds -2.1 % (profiles/r05/ord/)
template <uint32_t K>
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
  constexpr uint32_t row = K * kXcds;  // runs of K workgroups per XCD, the XCDs side by side
  const uint32_t full = nb / row * row;
  if (b >= full) return b;
  const uint32_t x = b % kXcds, i = b / kXcds;
  return i / K * row + x * K + i % K;
}

// Where a finished segment sum goes: a segment that continues into the next tile leaves its
// prefix in the next tile's crossing record for atmos_fixup_kernel; a complete one is the
// atmosphere value (and the boundary slot of a first/last atmosphere cell shared with a
// neighbour rank).
// R: the engine's output type (an fp32 engine's atmosphere outputs are float, rounded once)
template <class R>
__device__ __forceinline__ void segment_done(const AtmosFused &af, int64_t tile, int32_t a, const double *acc,
                                             bool cont) {
  if (cont) {  // the next tile's crossing record: the six prefix sums, 16-B stores
#pragma unroll
    for (int q = 0; q < kFusedFields / 2; ++q)
      gptr(reinterpret_cast<d2 *>(af.xrec + (tile + 1) * kXRec))[q] = d2{acc[2 * q], acc[2 * q + 1]};
    return;
  }
  if (FCX_DBG_ATM_NOSTORE) return;
// Non-temporal atmosphere-output stores for fp64 outputs.  Since the segment sums run in
// rounds, a round writes the tile's values of a field with one instruction, and for fp64
// outputs NT stores gained 3.4-4.4 % per step (periodic / random map); fp32 outputs lost 7 %
// with them, and NT only for the lines a tile owns whole changed nothing
// (profiles/r02/nt_atm_ab/; round 1, with one store instruction per cell position, all-NT
// had lost 6.8 %).
#pragma unroll
  for (int k = 0; k < kFusedFields; ++k) {
    if (!af.out[k]) continue;
    FCX_GLOBAL R *o = gptr(reinterpret_cast<R *>(af.out[k]) + tiled(a, af.out_tpad));
    if constexpr (sizeof(R) == 8)
      __builtin_nontemporal_store((R)acc[k], o);
    else
      *o = (R)acc[k];
    if (a == 0 && af.left >= 0) gptr(af.shared)[(int64_t)af.left * af.stride + af.scol[k]] = acc[k];
    if (a == af.n_atmos - 1 && af.right >= 0) gptr(af.shared)[(int64_t)af.right * af.stride + af.scol[k]] = acc[k];
  }
}

// blocks per CU the multi-type (RAVG) fused kernel is compiled for: 3 -> <= 168 VGPRs, room
// for the held atmosphere-side inputs (4 -> <= 128 spills them: T = 2 step +24 %).  2 gives
// the same 3 waves per SIMD (+1 VGPR): -0.7 % in one process over shared arrays, +0.5 % in
// alternating bench processes on one box (profiles/r03/ravg_blocks_ab/): 3 stays.
#ifndef FCX_RAVG_ATMOS_BLOCKS
#define FCX_RAVG_ATMOS_BLOCKS 3
#endif
// blocks per CU the T=1 fused kernels are compiled for (1: no register cap)
#ifndef FCX_T1_ATMOS_BLOCKS
#define FCX_T1_ATMOS_BLOCKS 1
#endif
// ... and the fp32 T=1 fused CCLM / MOM5 kernels (4 cells per lane): 4 = at most 128 VGPRs,
// 4 waves per SIMD, no spills (uncapped they take 132 / 137 VGPRs and 3 waves); in one
// process over the same arrays (profiles/r03/ab_f32_4waves.json) CCLM 4.81 -> 5.19 TB/s,
// MOM5 4.73 -> 5.08.  The fp32 RCO kernel (105 VGPRs, 4 waves either way) lost 5 % under the
// cap and keeps none.  1 (A/B): no cap.
#ifndef FCX_F32_ATMOS_BLOCKS
#define FCX_F32_ATMOS_BLOCKS 4
#endif
// waves per block of the fused kernel (A/B knobs)
#ifndef FCX_ATMOS_WAVES
#define FCX_ATMOS_WAVES 4
#endif
#ifndef FCX_F32_ATMOS_WAVES  // A/B: 2 paid while the fp32 rows held fp64 products (13.8 KB/wave)
#define FCX_F32_ATMOS_WAVES 4
#endif
template <int C>
constexpr int atmos_waves() { return C == 4 ? FCX_F32_ATMOS_WAVES : FCX_ATMOS_WAVES; }
// HALO (T = 1, full-range launches, maps whose segments are at most halo * C + 1 cells): a
// wave owns the first 64 - halo lanes' cells of its tile and computes the last `halo` lanes'
// cells -- the head of the next tile -- only for their products (nothing of them is stored),
// so every segment that starts in its own cells is summed inside the wave: no crossing
// records, no fix-up launch.  Tiles are (64 - halo) * C cells apart.
// One wave tile of the fused kernel: the fluxes of the tile's cells (process), their
// products w * x parked in the wave's LDS rows, the segment sums in rounds, the crossing
// record.  wp: the wave's LDS region.
template <int C, class R, int VAR, bool NT, int TM, bool RAVG, bool REC, bool HALO>
__device__ __forceinline__ void atmos_tile(const Params *__restrict__ P, const double *__restrict__ corr_m,
                                           const AtmosFused &af, int64_t tile, double *wp) {
  constexpr int kT = tile_cells<C>();  // cells per wave tile (lane l: cells C*l .. C*l+C-1)
  constexpr int kR = row_len<C>();
  constexpr bool kXF = sizeof(R) == 4;  // LDS holds fp32 fluxes + fp64 weights
  const int64_t n = P->n_max;
  const int own_lanes = HALO ? 64 - af.halo : 64;
  const int64_t kO = (int64_t)C * own_lanes;  // cells a tile owns (HALO: lo == 0)
  const int lane = threadIdx.x & 63;
  const uint64_t at_or_above = ~0ull << lane;
  const uint64_t above = lane == 63 ? 0ull : (~0ull << (lane + 1));
    const int64_t t0 = tile * kO;
    const int64_t j0 = t0 + C * lane;
    LdsEmitT<C> emit{wp, {}, lds_slot(C * lane)};
    // the lane's cells in the compacted map: which start a segment (cells past the grid end
    // count as starts: they end the last real segment) and, for those, the segment's
    // atmosphere cell; the lane's C cells share one bit word (j0 is a multiple of C)
    // fp32 and fp64 halo tiles (kCompact): the compacted map -- the bit word and prefix
    // count are loaded with the inputs, the dependent loads of the segments' atmosphere cells
    // follow the flux pass, so they add no round trip before it.  fp64 with crossing records:
    // one 4-B index per cell, loaded with the inputs (the compacted map measured -2.3 % per
    // fp32 step, -0.4 / -1.1 % at T = 1 fp64 and +1.7 % at T = 2 -- its records' first-cell
    // load is a fourth dependent one -- in one process over the same arrays: profiles/r05/seg/)
    constexpr bool kCompact = compact_map(sizeof(R) == 4, HALO);
    const int sh = (int)(j0 & 31);
    uint32_t word = 0;
    int32_t before = 0;  // kCompact: segments starting before cell j0
    int32_t a[C];        // atmosphere cell (kCompact: of a segment-start cell only; -1 elsewhere)
#pragma unroll
    for (int i = 0; i < C; ++i) a[i] = -1;
    int32_t a0_tile = 0;  // kCompact, crossing records: the tile's first cell's atmosphere cell
    if constexpr (kCompact) {
      if (j0 < n) {
        word = gptr(af.seg_bits)[j0 >> 5];
        before = gptr(af.seg_pre)[j0 >> 5];
      }
      if (!HALO && af.xrec_on) a0_tile = gptr(af.tile_a0)[tile];
    } else if (j0 + C <= n) {
      const i2v ii = *gptr(reinterpret_cast<const i2v *>(af.idx + j0));
      a[0] = ii.x;
      a[1] = ii.y;
    } else {
#pragma unroll
      for (int i = 0; i < C; ++i)
        if (j0 + i < n) a[i] = gptr(af.idx)[j0 + i];
    }
    if (j0 + C <= n) {
#pragma unroll
      for (int h = 0; h < C / 2; ++h) {
        const d2 ww = __builtin_nontemporal_load(gptr(reinterpret_cast<const d2 *>(af.w + j0) + h));
        emit.w[2 * h] = ww[0];
        emit.w[2 * h + 1] = ww[1];
      }
    } else {
#pragma unroll
      for (int i = 0; i < C; ++i)
        if (j0 + i < n) emit.w[i] = gptr(af.w)[j0 + i];
    }
    const int64_t tend = t0 + kT;
    // the segment running to the tile end continues past it (wave-uniform loads)
    bool next_cont;
    int32_t prev_tile = -2;
    if constexpr (kCompact) {
      next_cont = tend < n && !((gptr(af.seg_bits)[tend >> 5] >> (tend & 31)) & 1u);
    } else {
      prev_tile = t0 > 0 ? gptr(af.idx)[t0 - 1] : -2;
      next_cont = tend < n && gptr(af.idx)[tend] == gptr(af.idx)[tend - 1];
    }
    if (j0 < n)
      process<C, true, VAR, NT, R, TM, RAVG, LdsEmitT<C>, REC, HALO>(
          P, corr_m, j0, emit, AccLds<C, R>{reinterpret_cast<R *>(wp + emit.s), kR}, t0 + kO);
    if constexpr (kXF) {  // the weights row of the fp32 fluxes (dead cells: weight 0)
#pragma unroll
      for (int h = 0; h < C / 2; ++h)
        *reinterpret_cast<d2 *>(wp + xrows_doubles<C>() + emit.s + 2 * h) = d2{emit.w[2 * h], emit.w[2 * h + 1]};
    }
    // cell e of the tile added to a segment sum, in link order: its products w * x
    auto add_cell = [&](double *acc, int e) {
      if constexpr (kXF) {
        const float *xr = reinterpret_cast<const float *>(wp);
        const double we = wp[xrows_doubles<C>() + lds_slot(e)];
#pragma unroll
        for (int k = 0; k < kFusedFields; ++k) acc[k] = acc[k] + we * (double)xr[k * kT + e];
      } else {
        const double *q = wp + lds_slot(e);
#pragma unroll
        for (int k = 0; k < kFusedFields; ++k) acc[k] = acc[k] + q[k * kR];
      }
    };
    // segment starts: cell C*l+i begins a segment when its atmosphere cell differs from the
    // previous cell's (cells past the grid end also "start", which ends the last real segment)
    bool st[C];
    uint64_t m[C];
    if constexpr (kCompact) {
      before += __builtin_popcount(word & ((1u << sh) - 1u));
      int32_t ord = before;
#pragma unroll
      for (int i = 0; i < C; ++i) {
        const bool valid = j0 + i < n;
        st[i] = !valid || ((word >> (sh + i)) & 1u);
        if (valid && st[i]) a[i] = gptr(af.seg_atm)[ord++];
        m[i] = __ballot(st[i]);
      }
    } else {
      int32_t prev = __shfl_up(a[C - 1], 1);
      if (lane == 0) prev = prev_tile;
#pragma unroll
      for (int i = 0; i < C; ++i) {
        st[i] = a[i] != (i ? a[i - 1] : prev);
        m[i] = __ballot(st[i]);
      }
    }
    wave_sync();  // the wave's LDS products are visible to all its lanes
    // Rounds of one segment start per lane (round 2): every lane with a start sums its
    // segment and stores the six values in the same round, so a tile's atmosphere stores are
    // six store instructions per round (one round when every run is >= C cells long, as on an
    // intersection grid), not six per cell position of the lane as in round 1
    // (profiles/r02/seg_rounds_ab/).
    uint32_t rem = 0;  // bit i: cell C*lane+i starts a segment not summed yet (an own cell)
#pragma unroll
    for (int i = 0; i < C; ++i)
      if (st[i] && j0 + i < n && (!HALO || lane < own_lanes)) rem |= 1u << i;
    // the end of the segment starting at cell C*lane+i: the next start of any kind (own,
    // halo, past the grid end), or the tile end
    auto seg_end = [&](int i) {
      int e_end = kT;
#pragma unroll
      for (int q = 0; q < C; ++q) e_end = min(e_end, C * first_bit(m[q] & (q > i ? at_or_above : above)) + q);
      return min(e_end, kT);
    };
    // ... of the segment starting at any cell c of the tile (the lane summing it need not hold it)
    auto seg_end_of = [&](int c) {
      const int l = c / C, i = c % C;
      const uint64_t ge = ~0ull << l, gt = l == 63 ? 0ull : (~0ull << (l + 1));
      int e_end = kT;
#pragma unroll
      for (int q = 0; q < C; ++q) e_end = min(e_end, C * first_bit(m[q] & (q > i ? ge : gt)) + q);
      return min(e_end, kT);
    };
    if constexpr (seg_ordinal<R, C>()) {
      static_assert(kT == 256 && kSegCap * 8 == kT * 6, "one list entry per cell of the tile");
      uint16_t *seg = reinterpret_cast<uint16_t *>(wp + xrows_doubles<C>() + row_len<C>());  // [kT]
      int32_t *seg_a = reinterpret_cast<int32_t *>(seg + kT);                                 // [kT]
      const uint64_t lower = (1ull << lane) - 1;
      int total = 0, o = 0;  // the tile's segments; this lane's first one's ordinal
#pragma unroll
      for (int q = 0; q < C; ++q) {
        const uint64_t b = __ballot((rem >> q) & 1u);
        total += __popcll(b);
        o += __popcll(b & lower);
      }
#pragma unroll
      for (int i = 0; i < C; ++i)
        if ((rem >> i) & 1u) {
          seg[o] = (uint16_t)(C * lane + i);
          seg_a[o] = a[i];
          ++o;
        }
      wave_sync();
      for (int base = 0; base < total; base += 64) {
        const int sg = base + lane;
        if (sg < total) {
          const int c = seg[sg];
          const int end = seg_end_of(c);
          const int32_t ai = seg_a[sg];
          double acc[kFusedFields];
#pragma unroll
          for (int k = 0; k < kFusedFields; ++k) acc[k] = 0.0;
          for (int e = c; e < end; ++e) add_cell(acc, e);
          segment_done<R>(af, tile, ai, acc, !HALO && end == kT && next_cont);
        }
      }
      rem = 0;
    }
    while (__ballot(rem != 0)) {
      if (rem) {
        const int i = __builtin_ctz(rem);
        rem &= rem - 1;
        int32_t ai = a[0];
#pragma unroll
        for (int q = 1; q < C; ++q)
          if (q == i) ai = a[q];
        const int c = C * lane + i;
        // next start after cell c: cell C*j+i' with j > l, or j == l and i' > i
        const int end = seg_end(i);
        double acc[kFusedFields];
#pragma unroll
        for (int k = 0; k < kFusedFields; ++k) acc[k] = 0.0;
        for (int e = c; e < end; ++e) add_cell(acc, e);
        // (HALO: the segment ends inside the wave's own + halo cells by the engine's rule)
        segment_done<R>(af, tile, ai, acc, !HALO && end == kT && next_cont);
      }
    }
    // the number of head cells (continuing the previous tile's segment) for
    // atmos_fixup_kernel; 0 when the tile starts a segment
    if (!HALO && af.xrec_on) {  // (a map whose segments never cross a tile needs no records)
      int head = kT;
#pragma unroll
      for (int q = 0; q < C; ++q) head = min(head, C * first_bit(m[q]) + q);
      if (FCX_DBG_NO_HEAD >= 2) head = 0;
      double *xr0 = af.xrec + tile * kXRec;
      if (lane == 0 && FCX_DBG_NO_HEAD < 2) {  // the tile's first cell: its atmosphere cell
        const int32_t a0 = kCompact ? a0_tile : a[0];
        *gptr(reinterpret_cast<i2v *>(xr0 + 30)) = i2v{head, a0};
      }
      if (FCX_DBG_NO_HEAD) head = 0;
      // the products of the first kRecHead head cells, one lane per cell, 16-B stores
      if (lane < min(head, kRecHead)) {
        double hp[kFusedFields];
        if constexpr (kXF) {
          const float *xr = reinterpret_cast<const float *>(wp);
          const double we = wp[xrows_doubles<C>() + lds_slot(lane)];
#pragma unroll
          for (int k = 0; k < kFusedFields; ++k) hp[k] = we * (double)xr[k * kT + lane];
        } else {
#pragma unroll
          for (int k = 0; k < kFusedFields; ++k) hp[k] = wp[k * kR + lds_slot(lane)];
        }
#pragma unroll
        for (int q = 0; q < kFusedFields / 2; ++q)
          gptr(reinterpret_cast<d2 *>(xr0 + kFusedFields + lane * kFusedFields))[q] = d2{hp[2 * q], hp[2 * q + 1]};
      }
    }
    wave_sync();  // every lane is done reading before the next tile overwrites the region
}

template <int C, class R, int VAR, bool NT, int TM, bool RAVG, bool REC = false, bool HALO = false>
// (REC: the record stores took CCLM to 129 VGPRs and 3 waves per SIMD; capped at 4 blocks = 4 waves)
__global__ __launch_bounds__(64 * atmos_waves<C>(), RAVG  ? FCX_RAVG_ATMOS_BLOCKS
                                                  : REC ? 4
                                                  : (C == 4 && VAR != 3) ? FCX_F32_ATMOS_BLOCKS
                                                                         : FCX_T1_ATMOS_BLOCKS) void cells_atmos_kernel(const Params *__restrict__ P,
                                                          const double *__restrict__ corr_m,
                                                          const AtmosFused af, int64_t lo, int64_t hi) {
  static_assert(!RAVG || (C == 2 && sizeof(R) == 8), "register averages: fp64 engine only");
  static_assert(sizeof(R) == 8 || C == 4 || C == 2, "fp32 flux rows: 4 or 2 cells per lane");
  // product rows [kFusedFields][kR]; with RAVG they first serve as the accumulators of
  // the type-0 averages (slot k = row k, TSUR in an extra row), then hold w * average
  constexpr int kRows = RAVG ? kAvgSlots : kFusedFields;
  __shared__ double s_p[atmos_waves<C>()][wave_lds_doubles<R, C>(kRows)];
  static_assert(!HALO || (TM == 1 && !RAVG) || (FCX_HALO_RAVG && RAVG), "halo tiles: the T=1 launch");
  const int own_lanes = HALO ? 64 - af.halo : 64;
  const int64_t kO = (int64_t)C * own_lanes;  // cells a tile owns (HALO: lo == 0)
  const int64_t n_tiles = af.n_tiles;  // (hi + kO - 1) / kO, from the host
  const int wv = threadIdx.x >> 6;
  double *wp = s_p[wv];
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wave0 =
      (int64_t)xcd_block<C == 4 ? FCX_XCD_CHUNK_F32 : FCX_XCD_CHUNK>(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + wv;
#if FCX_WAVE_TRACE
  const int lane = threadIdx.x & 63;
  const uint64_t trace_start = (uint64_t)wall_clock64();
  uint64_t trace_loop = 0;
#endif
  for (int64_t tile = lo / kO + wave0; tile < n_tiles; tile += waves) {
#if FCX_WAVE_TRACE
    if (!trace_loop) trace_loop = (uint64_t)wall_clock64();
#endif
    atmos_tile<C, R, VAR, NT, TM, RAVG, REC, HALO>(P, corr_m, af, tile, wp);
  }
#if FCX_WAVE_TRACE
  if (af.trace) {
    __builtin_amdgcn_s_waitcnt(0);  // the wave's stores have completed
    const uint64_t trace_end = (uint64_t)wall_clock64();
    if (lane == 0) {
      const uint64_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      const uint64_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
      u64x2 *t = reinterpret_cast<u64x2 *>(af.trace + ((int64_t)blockIdx.x * (blockDim.x >> 6) + wv) * 4);
      t[0] = u64x2{trace_start, trace_end};
      t[1] = u64x2{hw | (xcc << 32), trace_loop};
    }
  }
#endif
}


// Several engines' fused launches as ONE launch (fcx_run_group): the members' wave
// tiles side by side in one grid, [member 0's tiles][member 1's]..., each wave running the
// tile of its member with that member's parameter block, variant and accumulation.  One
// launch instead of one per engine: the ramp-up and the drain tail of a launch (~20-25 us
// each) are paid once per step, and the tail of one member's tiles
// overlaps the next member's.  Per tile the same code as cells_atmos_kernel, so the same bits.
// Blocks per CU the fp64 T = 1 group kernel is compiled for: 4 = 128 VGPRs, 4 waves per SIMD
// like the members' own kernels (left free, the three inlined bodies take 139-146 VGPRs and
// 3 waves; at 128 one 8-B value of the preamble spills: one store and two reloads per wave).
// The multi-type group (RAVG) keeps the members' FCX_RAVG_ATMOS_BLOCKS.
#ifndef FCX_GROUP_BLOCKS
#define FCX_GROUP_BLOCKS 4
#endif
template <int C, class R, bool NT, bool HALO, int TM = 1, bool RAVG = false>
__global__ __launch_bounds__(64 * atmos_waves<C>(), RAVG ? FCX_RAVG_ATMOS_BLOCKS
                                                    : C == 4 ? FCX_F32_ATMOS_BLOCKS : FCX_GROUP_BLOCKS) void
cells_atmos_group_kernel(const GroupArgs g, const Params *__restrict__ P0, const Params *__restrict__ P1,
                         const Params *__restrict__ P2, const Params *__restrict__ P3) {
  // The members' parameter blocks are separate const __restrict__ kernel arguments (not the
  // pointers inside GroupArgs): the compiler then knows the blocks are not written by the
  // launch and reads them with scalar loads, as in cells_atmos_kernel.  Read through a
  // pointer out of the argument struct, every field was a vector load (and a dependent
  // round trip before the field loads): the group kernel took 1.156 ms against 0.783 ms
  // for the three launches it replaced (a round-4 diagnostic build, not kept).
  constexpr int kRows = RAVG ? kAvgSlots : kFusedFields;
  __shared__ double s_p[atmos_waves<C>()][wave_lds_doubles<R, C>(kRows)];
  const int wv = threadIdx.x >> 6;
  double *wp = s_p[wv];
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wave0 =
      (int64_t)xcd_block<C == 4 ? FCX_XCD_CHUNK_F32 : FCX_XCD_CHUNK>(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + wv;
  for (int64_t t = wave0; t < g.total_tiles; t += waves) {
    // the range and member of tile t: wave-uniform, said so to the compiler (readfirstlane),
    // so that their parameters are scalar loads -- derived from threadIdx.x >> 6, the index
    // would be taken for a per-lane value and every member field would occupy VGPRs
    int q = 0;
    for (int j = 1; j < g.n_ranges; ++j)
      if (t >= g.r[j].t0) q = j;
    q = __builtin_amdgcn_readfirstlane(q);
    const GroupRange &rg = g.r[q];
    const int k = __builtin_amdgcn_readfirstlane(rg.member);
    const GroupMember &m = g.m[k];
    const Params *__restrict__ P = k == 0 ? P0 : k == 1 ? P1 : k == 2 ? P2 : P3;
    const int64_t tile = t - rg.t0 + rg.first;
    switch (m.var) {
      case 1: atmos_tile<C, R, 1, NT, TM, RAVG, false, HALO>(P, m.corr_m, m.af, tile, wp); break;
      case 2: atmos_tile<C, R, 2, NT, TM, RAVG, false, HALO>(P, m.corr_m, m.af, tile, wp); break;
      default: atmos_tile<C, R, 3, NT, TM, RAVG, false, HALO>(P, m.corr_m, m.af, tile, wp); break;
    }
  }
}

// Segments that straddle a tile boundary: the launch leaves, in the crossing record of every tile t, the prefix sum of tile t-1's last
// segment, the number of head cells of tile t (cells that continue that segment) with their
// atmosphere cell, and the products of the first kRecHead of them; this kernel continues each
// carry over the head cells, one thread per (tile, field), in link order: the same bits as
// the in-launch sum.  Cells of a longer head are recomputed from the stored fluxes with the
// kernel's own operation (w * x, fp32 fluxes widened).
// Segments are at most half a tile (the fused path's rule), so a carry never spans a tile.
// field k of the segment across tile boundary t (tile t's crossing record)
template <class R, int kT>
__device__ __forceinline__ void fixup_one(const AtmosFused &af, int64_t t, int k) {
  // one crossing record (two lines) holds everything of the common case: every load issued
  // before the head count is known, one memory round trip.  (One thread per boundary with
  // the whole record in 16-B loads measured the same: profiles/r04/crossings/inproc3/.)
  const int64_t x0 = t * kT;
  const double *rec = af.xrec + t * kXRec;
  const int2 ha = *reinterpret_cast<const int2 *>(rec + 30);
  double acc = rec[k];
  double p[kRecHead];
#pragma unroll
  for (int e = 0; e < kRecHead; ++e) p[e] = rec[kFusedFields + e * kFusedFields + k];
  const int h = ha.x;
  const int32_t a = ha.y;
  if (h == 0) return;
#pragma unroll
  for (int e = 0; e < kRecHead; ++e)
    if (e < h) acc = acc + p[e];
  const R *xk = reinterpret_cast<const R *>(af.x[k]);
  for (int e = kRecHead; e < h; ++e) acc = acc + af.w[x0 + e] * (double)xk[tiled(x0 + e, af.tpad)];
  reinterpret_cast<R *>(af.out[k])[tiled(a, af.out_tpad)] = (R)acc;
  if (a == 0 && af.left >= 0) af.shared[(int64_t)af.left * af.stride + af.scol[k]] = acc;
  if (a == af.n_atmos - 1 && af.right >= 0) af.shared[(int64_t)af.right * af.stride + af.scol[k]] = acc;
}

template <class R, int kT>
__global__ __launch_bounds__(256) void atmos_fixup_kernel(const AtmosFused af, int64_t n_tiles) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t t = 1 + i / kFusedFields;
  const int k = (int)(i % kFusedFields);
  if (t >= n_tiles || !af.out[k]) return;
  fixup_one<R, kT>(af, t, k);
}

// The fix-ups of a group launch's members (fcx_run_group) as ONE launch: member m's
// (boundary, field) threads are [first[m], first[m + 1]).  Each dependent launch costs the
// step its predecessor's drain, the dispatch and the ramp on top of its work: in one process
// over the same arrays, T = 2 group step 1.560 against 1.566 ms with one fix-up launch per
// member, T = 1 without halo tiles 0.759 against 0.766 ms (profiles/r04/crossings/inproc1/).
template <class R, int kT>
__global__ __launch_bounds__(256) void atmos_fixup_group_kernel(const FixupGroup g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.first[g.n]) return;
  int m = 0;
  for (int q = 1; q < g.n; ++q)
    if (i >= g.first[q]) m = q;
  const int64_t j = i - g.first[m];
  const int64_t t = 1 + j / kFusedFields;
  const int k = (int)(j % kFusedFields);
  if (!g.af[m].out[k]) return;
  fixup_one<R, kT>(g.af[m], t, k);
}

// do_regridding (basic:463-522) as CSR-by-destination: row d holds the links with
// dst_index == d in their original link order, so the sequential sum from 0.0 reproduces
// the reference's scatter-add order exactly (bit-identical) without atomics.
// R = float: the single-precision build's REAL(4) arithmetic.
template <class R>
__global__ __launch_bounds__(256) void regrid_csr_kernel(const int32_t *__restrict__ row_ptr,
                                                         const int32_t *__restrict__ col,
                                                         const R *__restrict__ w,
                                                         const R *__restrict__ src,
                                                         R *__restrict__ dst, int64_t n_dst, int64_t tpad) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n_dst) return;
  R acc = R(0);
  for (int32_t k = row_ptr[d]; k < row_ptr[d + 1]; ++k) acc = acc + src[tiled(col[k], tpad)] * w[k];
  dst[tiled(d, tpad)] = acc;
}

// exchange -> atmosphere accumulation (SCRIP weight application of the type-0 fields).
// One thread per local atmosphere cell, 256 cells per block.  The block's exchange range
// [row_ptr[a0], row_ptr[a0 + 256]) is streamed through LDS in chunks of kAtmChunk cells:
// the whole block loads weights and fields with coalesced loads (16-B vectors of consecutive
// links when the links are the exchange cells in order, `vec`) and stores the
// products w*x per field, then every lane adds the products of its own segment in link
// order.  acc = acc + w*x from 0.0 in increasing link order is exactly the sequential
// weight application, so the result is bit-identical to it (no atomics, no tree order).
#ifndef FCX_ATM_CHUNK
#define FCX_ATM_CHUNK 512
#endif
constexpr int kAtmChunk = FCX_ATM_CHUNK;

// R: element type of the fields and outputs (float in the fp32 engine; the weights, the
// products and the sums are fp64 either way, and an fp32 output is rounded once).
template <class R>
__global__ __launch_bounds__(256) void atmos_kernel(const AtmosArgs a) {
  extern __shared__ double lds[];  // [nf][kAtmChunk] products
  const int64_t a0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t c = a0 + threadIdx.x;
  const int64_t a_end = min(a0 + (int64_t)blockDim.x, a.n_atmos);
  const int32_t K0 = a.row_ptr[a0], K1 = a.row_ptr[a_end];
  constexpr int V = 16 / sizeof(R);  // elements per 16-B vector (2 fp64, 4 fp32)
  using VecT = typename std::conditional<sizeof(R) == 8, d2, f4>::type;
  const int32_t n_links = a.vec ? a.row_ptr[a.n_atmos] : 0;
  const bool mine = c < a.n_atmos;
  const int32_t k_lo = mine ? a.row_ptr[c] : 0, k_hi = mine ? a.row_ptr[c + 1] : 0;
  double acc[kMaxAtmosFields];
#pragma unroll
  for (int f = 0; f < kMaxAtmosFields; ++f) acc[f] = 0.0;
  for (int32_t C0 = K0; C0 < K1; C0 += kAtmChunk) {
    const int32_t len = min(kAtmChunk, K1 - C0);
    __syncthreads();
    if (a.vec) {  // link k = exchange cell k: 16-B loads of V consecutive weights and fields
      const int32_t hi_k = C0 + len;
      for (int32_t v = (C0 & ~(V - 1)) + (int32_t)threadIdx.x * V; v < hi_k; v += (int32_t)blockDim.x * V) {
        const bool full = v + V <= n_links;  // v..v+V-1 share a layout tile (V divides it)
        double wv[V];
        if (full) {
#pragma unroll
          for (int h = 0; h < V / 2; ++h) {
            const d2 t = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(a.w + v) + h);
            wv[2 * h] = t[0];
            wv[2 * h + 1] = t[1];
          }
        } else {
#pragma unroll
          for (int i = 0; i < V; ++i) wv[i] = v + i < n_links ? a.w[v + i] : 0.0;
        }
        const int64_t xo = tiled(v, a.tpad);
        for (int f = 0; f < a.nf; ++f) {
          const R *xf = reinterpret_cast<const R *>(a.x[f]) + xo;
          R xv[V];
          if (full) {
            const VecT t = __builtin_nontemporal_load(reinterpret_cast<const VecT *>(xf));
#pragma unroll
            for (int i = 0; i < V; ++i) xv[i] = t[i];
          } else {
#pragma unroll
            for (int i = 0; i < V; ++i) xv[i] = v + i < n_links ? xf[i] : R(0);
          }
#pragma unroll
          for (int i = 0; i < V; ++i)
            if (v + i >= C0 && v + i < hi_k) lds[f * kAtmChunk + (v + i - C0)] = wv[i] * (double)xv[i];
        }
      }
    } else if (a.rec) {  // remap gather of packed records: nf values of a link in rec_p / V 16-B loads
      for (int32_t i = threadIdx.x; i < len; i += blockDim.x) {
        const int32_t k = C0 + i;
        const int32_t xi = __builtin_nontemporal_load(a.col + k);
        const double wk = __builtin_nontemporal_load(a.w + k);
        const VecT *r = reinterpret_cast<const VecT *>(reinterpret_cast<const R *>(a.rec) + (int64_t)xi * a.rec_p);
#pragma unroll
        for (int q = 0; q < kMaxAtmosFields / V; ++q) {
          if (q * V >= a.nf) break;
          const VecT t = r[q];
#pragma unroll
          for (int h = 0; h < V; ++h)
            if (q * V + h < a.nf) lds[(q * V + h) * kAtmChunk + i] = wk * (double)t[h];
        }
      }
    } else {
      for (int32_t i = threadIdx.x; i < len; i += blockDim.x) {
        const int32_t k = C0 + i;
        const int32_t xi = a.col ? a.col[k] : k;
        const double wk = __builtin_nontemporal_load(a.w + k);
#pragma unroll
        for (int f = 0; f < kMaxAtmosFields; ++f)
          if (f < a.nf) lds[f * kAtmChunk + i] = wk * (double)reinterpret_cast<const R *>(a.x[f])[tiled(xi, a.tpad)];
      }
    }
    __syncthreads();
    const int32_t lo = max(k_lo, C0), hi = min(k_hi, C0 + len);
    for (int32_t k = lo; k < hi; ++k) {
#pragma unroll
      for (int f = 0; f < kMaxAtmosFields; ++f)
        if (f < a.nf) acc[f] = acc[f] + lds[f * kAtmChunk + (k - C0)];
    }
  }
  if (!mine) return;
#pragma unroll
  for (int f = 0; f < kMaxAtmosFields; ++f) {
    if (f >= a.nf) break;
    reinterpret_cast<R *>(a.out[f])[tiled(c, a.out_tpad)] = (R)acc[f];
    if (c == 0 && a.left >= 0) a.shared[(int64_t)a.left * a.stride + a.scol[f]] = acc[f];
    if (c == a.n_atmos - 1 && a.right >= 0) a.shared[(int64_t)a.right * a.stride + a.scol[f]] = acc[f];
  }
}

// Remap records (row f3).  A remap link gathers the nf sent fields of one scattered exchange
// cell; from nf separate arrays that is nf scattered 8-B reads, each of which costs the
// memory a whole 32-B sector (PMC: 4x the algorithmic read bytes on a shuffled 2-link map).
// Packed cell-major, the nf values of a cell are one record of P = nf rounded up to 16 B,
// read by P / V 16-B loads that share its sectors.  One block packs 256 * V cells: the
// fields are staged in LDS with coalesced 16-B loads (the block's cells lie in one layout
// tile), then the block's contiguous record region is written with 16-B stores.
template <class R>
__global__ __launch_bounds__(256) void pack_records_kernel(const AtmosArgs a, int64_t n, int32_t flags, R *rec) {
  constexpr int V = 16 / sizeof(R);
  constexpr int CB = 256 * V;  // cells per block (divides kLayoutTile)
  using VecT = typename std::conditional<sizeof(R) == 8, d2, f4>::type;
  extern __shared__ unsigned char lds_raw[];
  R *lds = reinterpret_cast<R *>(lds_raw);  // [nf][CB]
  const int64_t c0 = (int64_t)blockIdx.x * CB;
  const int64_t cn = min((int64_t)CB, n - c0);
  const int t = threadIdx.x;
  for (int f = 0; f < a.nf; ++f) {
    const R *x = reinterpret_cast<const R *>(a.x[f]) + tiled(c0, a.tpad);
    const int64_t j = (int64_t)t * V;
    if ((flags & 1) && j + V <= cn) {  // 16-B aligned fields
      const VecT *p = reinterpret_cast<const VecT *>(x + j);
      const VecT v = (flags & 2) ? __builtin_nontemporal_load(p) : *p;  // not for host-mapped fields
#pragma unroll
      for (int h = 0; h < V; ++h) lds[f * CB + j + h] = v[h];
    } else {
#pragma unroll
      for (int h = 0; h < V; ++h)
        if (j + h < cn) lds[f * CB + j + h] = x[j + h];
    }
  }
  __syncthreads();
  const int P = a.rec_p;
  const int64_t nvec = cn * P / V;  // P is a multiple of V: a vector never spans two records
  VecT *out = reinterpret_cast<VecT *>(rec + c0 * P);
  for (int64_t q = t; q < nvec; q += 256) {
    const int64_t e = q * V;
    const int64_t cell = e / P;
    const int f0 = (int)(e - cell * P);
    VecT v;
#pragma unroll
    for (int h = 0; h < V; ++h) v[h] = f0 + h < a.nf ? lds[(f0 + h) * CB + cell] : R(0);
    __builtin_nontemporal_store(v, out + q);  // +1 % over plain stores (profiles/r02/remap/)
  }
}

// after the all-reduce: completed boundary sums back into the outputs, then every slot of
// this engine's region is zeroed for the next step (one block)
template <class R>
__global__ void atmos_finish_kernel(const AtmosArgs a, int32_t n_boundaries) {
  const int t = threadIdx.x;
  if (t < a.nf) {
    R *out = reinterpret_cast<R *>(a.out[t]);
    if (a.left >= 0) out[0] = (R)a.shared[(int64_t)a.left * a.stride + a.scol[t]];
    if (a.right >= 0) out[tiled(a.n_atmos - 1, a.out_tpad)] = (R)a.shared[(int64_t)a.right * a.stride + a.scol[t]];
  }
  __syncthreads();
  for (int64_t i = t; i < (int64_t)n_boundaries * a.stride; i += blockDim.x) a.shared[i] = 0.0;
}

// the finishes of several engines after one exchange, one block per engine (one launch: each
// launch is ~5 us on the step's critical path after the all-reduce)
template <class R>
__global__ void atmos_finish_group_kernel(const FinishGroup g) {
  const AtmosArgs &a = g.a[blockIdx.x];
  const int32_t n_boundaries = g.nb[blockIdx.x];
  const int t = threadIdx.x;
  if (t < a.nf) {
    R *out = reinterpret_cast<R *>(a.out[t]);
    if (a.left >= 0) out[0] = (R)a.shared[(int64_t)a.left * a.stride + a.scol[t]];
    if (a.right >= 0) out[tiled(a.n_atmos - 1, a.out_tpad)] = (R)a.shared[(int64_t)a.right * a.stride + a.scol[t]];
  }
  __syncthreads();
  for (int64_t i = t; i < (int64_t)n_boundaries * a.stride; i += blockDim.x) a.shared[i] = 0.0;
}

__global__ void zero_kernel(double *x, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) x[j] = 0.0;
}

static int grid_for(int64_t units, int max_blocks = 256 * 8) {
  // memory-bound grid-stride: enough waves to fill 256 CUs, capped (0 = one unit per thread)
  int64_t blocks = (units + 255) / 256;
  if (max_blocks > 0 && blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

template <int C, bool MERGED, int VAR, bool NT, class R, int TM, bool RAVG>
static void launch_one(int blocks, hipStream_t s, const Params *dp, const double *corr_m, int64_t lo,
                       int64_t hi) {
  hipLaunchKernelGGL((cells_kernel<C, MERGED, VAR, NT, R, TM, RAVG>), dim3(blocks), dim3(256), 0, s, dp,
                     corr_m, lo, hi);
}

template <int C, bool MERGED, int VAR, class R, int TM, bool RAVG>
static void launch_nt(bool nt, int blocks, hipStream_t s, const Params *dp, const double *corr_m,
                      int64_t lo, int64_t hi) {
  if (nt)
    launch_one<C, MERGED, VAR, true, R, TM, RAVG>(blocks, s, dp, corr_m, lo, hi);
  else
    launch_one<C, MERGED, VAR, false, R, TM, RAVG>(blocks, s, dp, corr_m, lo, hi);
}

template <int C, class R, int TM, bool RAVG>
static void launch_c(const LaunchConfig &lc, int blocks, hipStream_t s, const Params *dp,
                     const double *corr_m, int64_t lo, int64_t hi) {
  if (!lc.merged) {
    launch_nt<C, false, 0, R, TM, RAVG>(lc.nontemporal, blocks, s, dp, corr_m, lo, hi);
    return;
  }
  switch (lc.variant) {
    case 1: launch_nt<C, true, 1, R, TM, RAVG>(lc.nontemporal, blocks, s, dp, corr_m, lo, hi); break;
    case 2: launch_nt<C, true, 2, R, TM, RAVG>(lc.nontemporal, blocks, s, dp, corr_m, lo, hi); break;
    case 3: launch_nt<C, true, 3, R, TM, RAVG>(lc.nontemporal, blocks, s, dp, corr_m, lo, hi); break;
    default: launch_nt<C, true, 0, R, TM, RAVG>(lc.nontemporal, blocks, s, dp, corr_m, lo, hi); break;
  }
}

template <int VAR>
static void launch_rec(bool nt, int blocks, hipStream_t s, const Params *dp, const double *corr_m, int64_t lo,
                       int64_t hi) {
  if (nt)
    hipLaunchKernelGGL((cells_kernel<2, true, VAR, true, double, 1, false, true>), dim3(blocks), dim3(256), 0, s, dp,
                       corr_m, lo, hi);
  else
    hipLaunchKernelGGL((cells_kernel<2, true, VAR, false, double, 1, false, true>), dim3(blocks), dim3(256), 0, s, dp,
                       corr_m, lo, hi);
}

// type mode: one surface type (compile-time), several, several with register averages
template <int C, class R>
static void launch_r(const Params *hp, const LaunchConfig &lc, int blocks, hipStream_t s, const Params *dp,
                     const double *corr_m, int64_t lo, int64_t hi) {
  if (hp->num_types == 1)
    launch_c<C, R, 1, false>(lc, blocks, s, dp, corr_m, lo, hi);
  else if (lc.ravg)
    launch_c<C, R, 0, true>(lc, blocks, s, dp, corr_m, lo, hi);
  else
    launch_c<C, R, 0, false>(lc, blocks, s, dp, corr_m, lo, hi);
}

template <int C, class R, int VAR, int TM, bool RAVG, bool REC = false, bool HALO = false>
static void launch_atm(bool nt, int blocks, hipStream_t s, const Params *dp, const double *corr_m,
                       const AtmosFused &af, int64_t lo, int64_t hi) {
  if (nt)
    hipLaunchKernelGGL((cells_atmos_kernel<C, R, VAR, true, TM, RAVG, REC, HALO>), dim3(blocks),
                       dim3(64 * atmos_waves<C>()), 0, s, dp, corr_m, af, lo, hi);
  else
    hipLaunchKernelGGL((cells_atmos_kernel<C, R, VAR, false, TM, RAVG, REC, HALO>), dim3(blocks),
                       dim3(64 * atmos_waves<C>()), 0, s, dp, corr_m, af, lo, hi);
}

// fused accumulation: one surface type (its fluxes), or several with the type-0 averages in
// registers (what OASIS sends); several types without register averages are not fused
template <int VAR>
static int launch_atm_r(const Params *hp, const LaunchConfig &lc, int blocks, hipStream_t s, const Params *dp,
                        const double *corr_m, const AtmosFused &af, int64_t lo, int64_t hi) {
  const bool halo = lc.halo > 0;
  if (halo && ((hp->num_types != 1 && !(FCX_HALO_RAVG && lc.ravg)) || lo != 0)) return (int)hipErrorInvalidValue;
  if (hp->num_types == 1 && lc.f32) {  // fp32 engine: 4 cells per lane, T = 1 only
    if (halo)
      launch_atm<kF32Cpl, float, VAR, 1, false, false, true>(lc.nontemporal, blocks, s, dp, corr_m, af, lo, hi);
    else
      launch_atm<kF32Cpl, float, VAR, 1, false>(lc.nontemporal, blocks, s, dp, corr_m, af, lo, hi);
  } else if (lc.f32) {
    return (int)hipErrorInvalidValue;
  } else if (hp->num_types == 1 && lc.rec) {
    if (halo)
      launch_atm<2, double, VAR, 1, false, true, true>(lc.nontemporal, blocks, s, dp, corr_m, af, lo, hi);
    else
      launch_atm<2, double, VAR, 1, false, true>(lc.nontemporal, blocks, s, dp, corr_m, af, lo, hi);
  } else if (hp->num_types == 1) {
    if (halo)
      launch_atm<2, double, VAR, 1, false, false, true>(lc.nontemporal, blocks, s, dp, corr_m, af, lo, hi);
    else
      launch_atm<2, double, VAR, 1, false>(lc.nontemporal, blocks, s, dp, corr_m, af, lo, hi);
  }
  else if (lc.ravg) {
    if constexpr (FCX_HALO_RAVG) {
      if (halo) {
        launch_atm<2, double, VAR, 0, true, false, true>(lc.nontemporal, blocks, s, dp, corr_m, af, lo, hi);
        return 0;
      }
    }
    launch_atm<2, double, VAR, 0, true>(lc.nontemporal, blocks, s, dp, corr_m, af, lo, hi);
  } else
    return (int)hipErrorInvalidValue;
  return 0;
}

#if FCX_WAVE_TRACE
// measurement builds: launch k of the fused kernel writes its wave timestamps into slot
// k % slots of a device buffer of slots x stride words (bench/wave_trace.py)
static struct {
  uint64_t *base = nullptr;
  int64_t stride = 0;
  int64_t slots = 1;
  int64_t launches = 0;
} g_trace;
}  // namespace fcx
extern "C" int fcx_debug_wave_trace(uint64_t *base, int64_t stride_words, int64_t slots, int64_t *wall_khz) {
  fcx::g_trace.base = base;
  fcx::g_trace.stride = stride_words;
  fcx::g_trace.slots = slots > 0 ? slots : 1;
  fcx::g_trace.launches = 0;
  int rate = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
    return 1;
  if (wall_khz) *wall_khz = rate;
  return 0;
}
namespace fcx {
#endif

int launch_cells(const Params *hp, const Params *dp, const double *corr_m, const LaunchConfig &lc,
                 void *stream, const AtmosFused *atm) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t lo = lc.lo, hi = lc.hi < 0 ? hp->n_max : std::min<int64_t>(lc.hi, hp->n_max);
  if (lo % kChunkAlign || lo < 0) return (int)hipErrorInvalidValue;
  if (hi <= lo) return 0;
  AtmosFused afl;  // this launch's copy: its tile count (and, in trace builds, its trace slot)
  if (atm) {
    afl = *atm;
    const int64_t own = (lc.f32 ? kF32Cpl : 2) * (64 - lc.halo);
    afl.n_tiles = (hi + own - 1) / own;
#if FCX_WAVE_TRACE
    afl.trace = g_trace.base ? g_trace.base + (g_trace.launches++ % g_trace.slots) * g_trace.stride : nullptr;
#endif
    atm = &afl;
  }
  if (atm) {  // fused accumulation: T=1 specialised merged kernel, 2 cells per lane
    // four waves per block (fp32: two), one 128-cell (fp32: 256-cell) tile per wave and trip.  Default: one trip (full
    // grid) -- +2 % per T=1 step over the 8192-block cap, equal at T=2 (profiles/r01/grid_ab)
    const int64_t kt = (lc.f32 ? kF32Cpl : 2) * (64 - lc.halo);  // cells a wave tile owns
    const int64_t kw = lc.f32 ? atmos_waves<kF32Cpl>() : atmos_waves<2>();
    const int64_t tiles = (hi - lo + kt - 1) / kt;
    const int64_t full = (tiles + kw - 1) / kw;
    const int blocks = (int)std::max<int64_t>(1, lc.max_blocks > 0 ? std::min<int64_t>(full, lc.max_blocks) : full);
    int r = 0;
    switch (lc.variant) {
      case 1: r = launch_atm_r<1>(hp, lc, blocks, s, dp, corr_m, *atm, lo, hi); break;
      case 2: r = launch_atm_r<2>(hp, lc, blocks, s, dp, corr_m, *atm, lo, hi); break;
      case 3: r = launch_atm_r<3>(hp, lc, blocks, s, dp, corr_m, *atm, lo, hi); break;
      default: return (int)hipErrorInvalidValue;
    }
    if (r) return r;
    return (int)hipGetLastError();
  }
  // vector width: 16 B per lane and array (2 fp64 or 4 fp32 cells), or 1 cell when the
  // caller's arrays are not 16-B aligned
  const int c = lc.cells_per_thread == 1 ? 1 : lc.f32 ? 4 : 2;
  const int64_t units = (hi - lo + c - 1) / c;
  const int blocks = grid_for(units, lc.max_blocks < 0 ? 8192 : lc.max_blocks);
  if (lc.rec) {  // remap records: the T=1 specialised fp64 kernels only (the planner's rule)
    if (lc.f32 || c != 2 || hp->num_types != 1 || !lc.merged || lc.variant < 1 || lc.variant > 3)
      return (int)hipErrorInvalidValue;
    switch (lc.variant) {
      case 1: launch_rec<1>(lc.nontemporal, blocks, s, dp, corr_m, lo, hi); break;
      case 2: launch_rec<2>(lc.nontemporal, blocks, s, dp, corr_m, lo, hi); break;
      default: launch_rec<3>(lc.nontemporal, blocks, s, dp, corr_m, lo, hi); break;
    }
    return (int)hipGetLastError();
  }
  if (lc.f32) {
    if (c == 4)
      launch_r<4, float>(hp, lc, blocks, s, dp, corr_m, lo, hi);
    else
      launch_r<1, float>(hp, lc, blocks, s, dp, corr_m, lo, hi);
  } else if (c == 2) {
    launch_r<2, double>(hp, lc, blocks, s, dp, corr_m, lo, hi);
  } else {
    launch_r<1, double>(hp, lc, blocks, s, dp, corr_m, lo, hi);
  }
  return (int)hipGetLastError();
}

template <int C, class R, bool NT>
static void launch_group_h(bool halo, bool ravg, int blocks, hipStream_t s, const GroupArgs &g) {
  const Params *p[kMaxGroup];
  for (int k = 0; k < kMaxGroup; ++k) p[k] = g.m[k < g.n ? k : 0].P;
  if constexpr (C == 2 && sizeof(R) == 8) {
    if (ravg) {  // several surface types, the type-0 averages in registers (no halo tiles)
      hipLaunchKernelGGL((cells_atmos_group_kernel<C, R, NT, false, 0, true>), dim3(blocks),
                         dim3(64 * atmos_waves<C>()), 0, s, g, p[0], p[1], p[2], p[3]);
      return;
    }
  }
  if (halo)
    hipLaunchKernelGGL((cells_atmos_group_kernel<C, R, NT, true>), dim3(blocks), dim3(64 * atmos_waves<C>()), 0, s, g,
                       p[0], p[1], p[2], p[3]);
  else
    hipLaunchKernelGGL((cells_atmos_group_kernel<C, R, NT, false>), dim3(blocks), dim3(64 * atmos_waves<C>()), 0, s,
                       g, p[0], p[1], p[2], p[3]);
}

int launch_cells_group(GroupMember *members, int n, const LaunchConfig &lc, void *stream) {
  if (n < 1 || n > kMaxGroup) return (int)hipErrorInvalidValue;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GroupArgs g{};
  g.n = n;
  int64_t total = 0;
  for (int k = 0; k < n; ++k) {  // (af.n_tiles: set by the caller from the member's cells)
    GroupMember &m = members[k];
    if (m.var < 1 || m.var > 3 || (m.af.halo > 0) != (lc.halo > 0) || m.af.n_tiles < 0)
      return (int)hipErrorInvalidValue;
    m.tile0 = total;
    g.m[k] = m;
    g.r[k] = GroupRange{total, 0, k, 0};
    total += m.af.n_tiles;
  }
  g.n_ranges = n;
  g.total_tiles = total;
  if (total == 0) return 0;
  const int64_t kw = lc.f32 ? atmos_waves<kF32Cpl>() : atmos_waves<2>();
  const int blocks = (int)std::max<int64_t>(1, (total + kw - 1) / kw);
  if (lc.ravg && (lc.f32 || lc.halo > 0)) return (int)hipErrorInvalidValue;
  if (lc.f32) {
    if (lc.nontemporal) launch_group_h<kF32Cpl, float, true>(lc.halo > 0, false, blocks, s, g);
    else launch_group_h<kF32Cpl, float, false>(lc.halo > 0, false, blocks, s, g);
  } else {
    if (lc.nontemporal) launch_group_h<2, double, true>(lc.halo > 0, lc.ravg, blocks, s, g);
    else launch_group_h<2, double, false>(lc.halo > 0, lc.ravg, blocks, s, g);
  }
  return (int)hipGetLastError();
}

int launch_regrid_csr(const int32_t *row_ptr, const int32_t *col, const double *w,
                      const double *src, double *dst, int64_t n_dst, void *stream, bool f32, int64_t tpad) {
  if (n_dst <= 0) return 0;
  const int blocks = (int)((n_dst + 255) / 256);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (f32)
    hipLaunchKernelGGL(regrid_csr_kernel<float>, dim3(blocks), dim3(256), 0, s, row_ptr, col,
                       reinterpret_cast<const float *>(w), reinterpret_cast<const float *>(src),
                       reinterpret_cast<float *>(dst), n_dst, tpad);
  else
    hipLaunchKernelGGL(regrid_csr_kernel<double>, dim3(blocks), dim3(256), 0, s, row_ptr, col, w, src, dst, n_dst, tpad);
  return (int)hipGetLastError();
}

int launch_atmos(const AtmosArgs &a, void *stream) {
  if (a.n_atmos <= 0 || a.nf <= 0) return 0;
  const int blocks = (int)((a.n_atmos + 255) / 256);
  const size_t lds = (size_t)a.nf * kAtmChunk * sizeof(double);
  if (a.f32)
    hipLaunchKernelGGL(atmos_kernel<float>, dim3(blocks), dim3(256), lds, reinterpret_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL(atmos_kernel<double>, dim3(blocks), dim3(256), lds, reinterpret_cast<hipStream_t>(stream), a);
  return (int)hipGetLastError();
}

int launch_pack_records(const AtmosArgs &a, int64_t n, bool aligned16, bool nontemporal, void *rec, void *stream) {
  if (n <= 0 || a.nf <= 0) return 0;
  const int V = a.f32 ? 4 : 2;
  if (a.rec_p < a.nf || a.rec_p % V || a.nf > kMaxAtmosFields) return (int)hipErrorInvalidValue;
  const int64_t cb = 256 * V;
  const int blocks = (int)((n + cb - 1) / cb);
  const size_t lds = (size_t)a.nf * cb * (a.f32 ? 4 : 8);
  const int32_t flags = (aligned16 ? 1 : 0) | (nontemporal ? 2 : 0);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a.f32)
    hipLaunchKernelGGL(pack_records_kernel<float>, dim3(blocks), dim3(256), lds, s, a, n, flags,
                       reinterpret_cast<float *>(rec));
  else
    hipLaunchKernelGGL(pack_records_kernel<double>, dim3(blocks), dim3(256), lds, s, a, n, flags,
                       reinterpret_cast<double *>(rec));
  return (int)hipGetLastError();
}

int launch_atmos_finish(const AtmosArgs &a, int32_t n_boundaries, void *stream) {
  if (!a.shared) return 0;
  if (a.f32)
    hipLaunchKernelGGL(atmos_finish_kernel<float>, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       a, n_boundaries);
  else
    hipLaunchKernelGGL(atmos_finish_kernel<double>, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       a, n_boundaries);
  return (int)hipGetLastError();
}

int launch_atmos_finish_group(const AtmosArgs *as, const int32_t *nbs, int n, void *stream) {
  if (n < 1 || n > kMaxGroup) return (int)hipErrorInvalidValue;
  FinishGroup g{};
  g.n = n;
  for (int k = 0; k < n; ++k) {
    if (!as[k].shared || as[k].f32 != as[0].f32) return (int)hipErrorInvalidValue;
    g.a[k] = as[k];
    g.nb[k] = nbs[k];
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (as[0].f32)
    hipLaunchKernelGGL(atmos_finish_group_kernel<float>, dim3(n), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(atmos_finish_group_kernel<double>, dim3(n), dim3(256), 0, s, g);
  return (int)hipGetLastError();
}

int launch_atmos_fixup(const AtmosFused &af, int64_t n, bool f32, void *stream) {
  const int64_t kt = f32 ? tile_cells<kF32Cpl>() : tile_cells<2>();
  const int64_t tiles = (n + kt - 1) / kt;
  if (tiles < 2) return 0;
  const int blocks = (int)(((tiles - 1) * kFusedFields + 255) / 256);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (f32)
    hipLaunchKernelGGL((atmos_fixup_kernel<float, tile_cells<kF32Cpl>()>), dim3(blocks), dim3(256), 0, s, af, tiles);
  else
    hipLaunchKernelGGL((atmos_fixup_kernel<double, tile_cells<2>()>), dim3(blocks), dim3(256), 0, s, af, tiles);
  return (int)hipGetLastError();
}

// Atmosphere cells without exchange cells: the sequential SCRIP sum over no links is 0, and
// the fused launch, which stores one value per segment, has none for them.
template <class R>
__global__ __launch_bounds__(256) void atmos_zero_kernel(const AtmosFused af, const int32_t *cells, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t a = cells[i];
#pragma unroll
  for (int k = 0; k < kFusedFields; ++k)
    if (af.out[k]) reinterpret_cast<R *>(af.out[k])[tiled(a, af.out_tpad)] = R(0);
}

int launch_atmos_zero(const AtmosFused &af, const int32_t *cells, int64_t n, bool f32, void *stream) {
  if (n <= 0) return 0;
  const int blocks = (int)((n + 255) / 256);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (f32)
    hipLaunchKernelGGL(atmos_zero_kernel<float>, dim3(blocks), dim3(256), 0, s, af, cells, n);
  else
    hipLaunchKernelGGL(atmos_zero_kernel<double>, dim3(blocks), dim3(256), 0, s, af, cells, n);
  return (int)hipGetLastError();
}

int launch_atmos_fixup_group(const AtmosFused *afs, const int64_t *n_cells, int n, bool f32, void *stream) {
  if (n < 1 || n > kMaxGroup) return (int)hipErrorInvalidValue;
  const int64_t kt = f32 ? tile_cells<kF32Cpl>() : tile_cells<2>();
  FixupGroup g{};
  g.n = n;
  for (int m = 0; m < n; ++m) {
    g.af[m] = afs[m];
    const int64_t tiles = (n_cells[m] + kt - 1) / kt;
    g.first[m + 1] = g.first[m] + std::max<int64_t>(tiles - 1, 0) * kFusedFields;
  }
  if (g.first[n] == 0) return 0;
  const int blocks = (int)((g.first[n] + 255) / 256);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (f32)
    hipLaunchKernelGGL((atmos_fixup_group_kernel<float, tile_cells<kF32Cpl>()>), dim3(blocks), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((atmos_fixup_group_kernel<double, tile_cells<2>()>), dim3(blocks), dim3(256), 0, s, g);
  return (int)hipGetLastError();
}

int launch_zero(double *x, int64_t n, void *stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(zero_kernel, dim3(grid_for(n)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, n);
  return (int)hipGetLastError();
}

}  // namespace fcx
