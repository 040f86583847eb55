// fcx_physics.h -- per-cell flux formulas of the reference flux_lib, as CDNA4 device code.
//
// Every literal is the double value of the reference's decimal text (the production build
// uses -r8, build_hlrnb.sh:26, so `17.2693882` is a REAL(8) constant) and every expression
// keeps the Fortran left-to-right evaluation order.  The translation unit is compiled
// with -ffp-contract=off so no FMA is formed: results differ from the reference only
// through the last-ulp behaviour of exp/pow (ROCm ocml vs glibc).
#pragma once
#include <hip/hip_runtime.h>

namespace fcx {

// flux_lib/constants/flux_constants.F90:13-32
constexpr double kCp = 1005.0;
constexpr double kLv = 2.501e6;
constexpr double kLs = 2.835e6;
constexpr double kRd = 287.05;
constexpr double kRv = 461.51;
constexpr double kSigma = 5.67e-8;
constexpr double kUmin = 0.01;

// flux_lib/auxiliaries/flux_aux_vapor.F90:20-70 (spec_vapor_surface_cclm)
__device__ __forceinline__ double qsur_cclm(double fice, double ps, double ts) {
  constexpr double aw = 17.2693882, ai = 21.8745584, t1 = 273.16, t2w = 35.86, t2i = 7.66,
                   p0 = 610.78;
  const double alpha = aw + (ai - aw) * fice;
  const double t2 = t2w + (t2i - t2w) * fice;
  const double e = p0 * exp(alpha * (ts - t1) / (ts - t2));
  return (kRd / kRv) * e / (ps - (1.0 - kRd / kRv) * e);
}

// T_tilde and the wind speed, shared by mass/heat/momentum (e.g. flux_mass_evap.F90:72-76)
__device__ __forceinline__ double t_tilde(double ts, double q) {
  return ts * (1.0 + (kRv / kRd - 1.0) * q);
}
__device__ __forceinline__ double wind(double u, double v) { return sqrt(u * u + v * v); }

// flux_lib/mass/flux_mass_evap.F90:72-83 (flux_mass_evap_cclm; _mom5 = same with CMOI)
__device__ __forceinline__ double meva_cclm(double a, double ps, double qa, double qs, double ts,
                                            double vel) {
  const double fa = a * fmax(vel, kUmin) * ps / (kRd * t_tilde(ts, qs));
  return fa * (qs - qa);
}

// flux_lib/mass/flux_mass_evap.F90:117-156 (flux_mass_evap_rco)
__device__ __forceinline__ double meva_rco(double qa, double ts, double vel) {
  constexpr double rho_a = 1.225, c_aw = 1.15E-03, eps = 0.62197, p_0 = 1.013E+05,
                   r = 6.1078E+02, c_1 = 17.269, c_2 = 35.86;
  const double e_w = r * exp(c_1 * (ts - 273.15) / (ts - c_2));
  const double q_w = eps * e_w / p_0;
  return rho_a * c_aw * vel * (q_w - qa);
}

// flux_lib/heat/flux_heat_sensible.F90:74-94 (flux_heat_sensible_cclm; _mom5 = with CHEA)
__device__ __forceinline__ double hsen_cclm(double a, double pa, double ps, double qs, double ta,
                                            double ts, double vel) {
  const double fa = a * fmax(vel, kUmin) * ps / (kRd * t_tilde(ts, qs));
  const double ef = pow(ps / pa, kRd / kCp);
  return fa * kCp * (ts - ta * ef);
}

// flux_lib/heat/flux_heat_sensible.F90:136-165 (flux_heat_sensible_rco)
__device__ __forceinline__ double hsen_rco(double ta, double ts, double vel) {
  constexpr double rho_a = 1.225, c_pa = 1.008E+03;
  const double c_aw = (ta < ts) ? 1.13E-03 : 0.66E-03;
  return rho_a * c_pa * c_aw * vel * (ts - ta);
}

// flux_lib/momentum/flux_momentum.F90:56-69: mass exchange rate; east = -(fa*u), north = -(fa*v)
__device__ __forceinline__ double mom_cclm_rate(double a, double ps, double qs, double ts,
                                                double vel) {
  return a * vel * ps / (kRd * t_tilde(ts, qs));
}

// flux_lib/momentum/flux_momentum.F90:107-136: -(rho_a*c_aw*vel*u) = -(rate*u)
__device__ __forceinline__ double mom_rco_rate(double vel) {
  constexpr double rho_a = 1.225;
  const double c_aw = (vel < 11.0) ? 1.2E-03 : 0.49E-03 + 0.065E-03 * vel;
  return rho_a * c_aw * vel;
}

// flux_lib/radiation/flux_radiation_blackbody.F90:22-42: sigma * T**4, lowered as
// ((T*T)*T)*T by the reference compiler
__device__ __forceinline__ double rbbr_stbo(double ts) { return kSigma * (ts * ts * ts * ts); }

}  // namespace fcx
