// fcx_physics.h -- per-cell flux formulas of the reference flux_lib, as CDNA4 device code.
//
// Every literal is the double value of the reference's decimal text (the production build
// uses -r8, build_hlrnb.sh:26, so `17.2693882` is a REAL(8) constant) and every expression
// keeps the Fortran left-to-right evaluation order.  The translation unit is compiled
// with -ffp-contract=off so no FMA is formed: in double the results differ from the
// reference only through the last-ulp behaviour of exp/pow (ROCm ocml vs glibc).
//
// R is the arithmetic type: double (the reference semantics) or float (the fp32 variant of
// fp32 storage and arithmetic, constants folded in double and then
// rounded once).  For R = double every expression is the one of the double-only code.
#pragma once
#include <hip/hip_runtime.h>

#include "fcx_internal.h"

namespace fcx {

// FCX_TRIVIAL_MATH=1 (A/B measurement builds only, FCX_AB_BUILD, never the product; see
// fcx_internal.h): every formula returns a plain sum of its inputs, so the kernels keep their
// loads, stores and accumulation but lose the fp64 exp/log/sqrt/division work -- the
// streaming ceiling of the kernel's own structure.
#define FCX_TRIVIAL(...)            \
  if constexpr (FCX_TRIVIAL_MATH) {   \
    return __VA_ARGS__;               \
  }

// flux_lib/constants/flux_constants.F90:13-32
constexpr double kCp = 1005.0;
constexpr double kLv = 2.501e6;
constexpr double kLs = 2.835e6;
constexpr double kRd = 287.05;
constexpr double kRv = 461.51;
constexpr double kSigma = 5.67e-8;
constexpr double kUmin = 0.01;

// flux_lib/auxiliaries/flux_aux_vapor.F90:20-70 (spec_vapor_surface_cclm)
template <class R>
__device__ __forceinline__ R qsur_cclm(R fice, R ps, R ts) {
  FCX_TRIVIAL(fice + ps + ts)
  constexpr R aw = R(17.2693882), ai = R(21.8745584), t1 = R(273.16), t2w = R(35.86),
              t2i = R(7.66), p0 = R(610.78);
  const R alpha = aw + (ai - aw) * fice;
  const R t2 = t2w + (t2i - t2w) * fice;
  const R e = p0 * exp(alpha * (ts - t1) / (ts - t2));
  return R(kRd / kRv) * e / (ps - R(1.0 - kRd / kRv) * e);
}

// T_tilde and the wind speed, shared by mass/heat/momentum (e.g. flux_mass_evap.F90:72-76)
template <class R>
__device__ __forceinline__ R t_tilde(R ts, R q) {
  return ts * (R(1) + R(kRv / kRd - 1.0) * q);
}
template <class R>
__device__ __forceinline__ R wind(R u, R v) {
  FCX_TRIVIAL(u + v)
  return sqrt(u * u + v * v);
}

// The atmosphere-only leading factor a * max(vel, u_min) * p_s of the CCLM/MOM5 exchange rate
// (flux_mass_evap.F90:76, flux_heat_sensible.F90:88), left to right as the reference
// evaluates it.  With several surface types and an atmosphere-side coefficient (CCLM: AMOI)
// the multi-type kernels form it once per cell; the formulas below are written through it,
// so both ways are the same operations and the same bits.
template <class R>
__device__ __forceinline__ R rate_num(R a, R vel, R ps) {
  return a * fmax(vel, R(kUmin)) * ps;
}

// flux_lib/mass/flux_mass_evap.F90:72-83 (flux_mass_evap_cclm; _mom5 = same with CMOI)
template <class R>
__device__ __forceinline__ R meva_cclm_num(R num, R qa, R qs, R ts) {
  const R fa = num / (R(kRd) * t_tilde(ts, qs));
  return fa * (qs - qa);
}
template <class R>
__device__ __forceinline__ R meva_cclm(R a, R ps, R qa, R qs, R ts, R vel) {
  FCX_TRIVIAL(a + ps + qa + qs + ts + vel)
  return meva_cclm_num(rate_num(a, vel, ps), qa, qs, ts);
}

// flux_lib/mass/flux_mass_evap.F90:117-156 (flux_mass_evap_rco)
template <class R>
__device__ __forceinline__ R meva_rco(R qa, R ts, R vel) {
  FCX_TRIVIAL(qa + ts + vel)
  constexpr R rho_a = R(1.225), c_aw = R(1.15E-03), eps = R(0.62197), p_0 = R(1.013E+05),
              r = R(6.1078E+02), c_1 = R(17.269), c_2 = R(35.86);
  const R e_w = r * exp(c_1 * (ts - R(273.15)) / (ts - c_2));
  const R q_w = eps * e_w / p_0;
  return rho_a * c_aw * vel * (q_w - qa);
}

// x**y for the Exner ratio ps/pa (within a few percent of 1) and y = Rd/cp: exp(y * log x).
// With |y log x| < 0.01 the argument's error is ~1e-19 relative, so the result is as close
// to x**y as a library pow (last-ulp differences only, like the reference's own pow against
// ROCm's), at a fraction of ROCm's fp64 pow, which carries extra-precision log/exp for any
// base.  Special values agree with pow for y > 0 (0 -> 0, inf -> inf, x < 0 or NaN -> NaN).
#ifndef FCX_POW_EXPLOG
#define FCX_POW_EXPLOG 1
#endif
template <class R>
__device__ __forceinline__ R pow_exner(R x, R y) {
#if FCX_POW_EXPLOG
  return exp(y * log(x));
#else
  return pow(x, y);
#endif
}

// flux_lib/heat/flux_heat_sensible.F90:74-94 (flux_heat_sensible_cclm; _mom5 = with CHEA).
// T_a * EF = T_a * (p_s / p_a)**(R_d / c_p) involves atmosphere fields only: the multi-type
// kernels form it once per cell (ta_exner) instead of one pow per surface type.
template <class R>
__device__ __forceinline__ R ta_exner(R ta, R ps, R pa) {
  return ta * pow_exner(ps / pa, R(kRd / kCp));
}
template <class R>
__device__ __forceinline__ R hsen_cclm_num(R num, R qs, R ts, R taef) {
  const R fa = num / (R(kRd) * t_tilde(ts, qs));
  return fa * R(kCp) * (ts - taef);
}
template <class R>
__device__ __forceinline__ R hsen_cclm(R a, R pa, R ps, R qs, R ta, R ts, R vel) {
  FCX_TRIVIAL(a + pa + ps + qs + ta + ts + vel)
  return hsen_cclm_num(rate_num(a, vel, ps), qs, ts, ta_exner(ta, ps, pa));
}

// flux_lib/heat/flux_heat_sensible.F90:136-165 (flux_heat_sensible_rco)
template <class R>
__device__ __forceinline__ R hsen_rco(R ta, R ts, R vel) {
  FCX_TRIVIAL(ta + ts + vel)
  constexpr R rho_a = R(1.225), c_pa = R(1.008E+03);
  const R c_aw = (ta < ts) ? R(1.13E-03) : R(0.66E-03);
  return rho_a * c_pa * c_aw * vel * (ts - ta);
}

// flux_lib/momentum/flux_momentum.F90:56-69: mass exchange rate; east = -(fa*u), north = -(fa*v)
// (no u_min here); a * vel * p_s is atmosphere-only for CCLM (AMOM): mom_num, formed once
template <class R>
__device__ __forceinline__ R mom_num(R a, R vel, R ps) {
  return a * vel * ps;
}
template <class R>
__device__ __forceinline__ R mom_cclm_rate_num(R num, R qs, R ts) {
  return num / (R(kRd) * t_tilde(ts, qs));
}
template <class R>
__device__ __forceinline__ R mom_cclm_rate(R a, R ps, R qs, R ts, R vel) {
  FCX_TRIVIAL(a + ps + qs + ts + vel)
  return mom_cclm_rate_num(mom_num(a, vel, ps), qs, ts);
}

// flux_lib/momentum/flux_momentum.F90:107-136: -(rho_a*c_aw*vel*u) = -(rate*u)
template <class R>
__device__ __forceinline__ R mom_rco_rate(R vel) {
  FCX_TRIVIAL(vel + vel)
  constexpr R rho_a = R(1.225);
  const R c_aw = (vel < R(11.0)) ? R(1.2E-03) : R(0.49E-03) + R(0.065E-03) * vel;
  return rho_a * c_aw * vel;
}

// flux_lib/radiation/flux_radiation_blackbody.F90:22-42: sigma * T**4, lowered as
// ((T*T)*T)*T by the reference compiler
template <class R>
__device__ __forceinline__ R rbbr_stbo(R ts) {
  return R(kSigma) * (ts * ts * ts * ts);
}

}  // namespace fcx
