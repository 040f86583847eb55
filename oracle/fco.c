/*
 * fco.c -- CPU ORACLE (plain C restatement) of the reference flux path.
 * TEST INFRASTRUCTURE ONLY: see fco.h.  Never linked into the product.
 *
 * Every formula below restates the reference Fortran with -r8 semantics (all decimal
 * literals are doubles, build_hlrnb.sh:23,26) and the exact left-to-right evaluation
 * order of the Fortran expression.  Built with -ffp-contract=off so no FMA is formed,
 * matching the reference DEBUG build (-fp-model precise).  It is pinned bit-for-bit
 * against oracle/_ref (the reference flux_lib compiled from /root/reference sources)
 * by tests/test_oracle_golden.py.
 */
#include "fco.h"
#include <math.h>
#include <string.h>
#include <stddef.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* flux_constants.F90:13-32 (default_values) */
static const double C_P = 1005.0, L_V = 2.501e6, L_S = 2.835e6;
static const double R_D = 287.05, R_V = 461.51, SIGMA = 5.67e-8, U_MIN = 0.01;

/* ---------------- per-cell formulas (flux_lib) ---------------- */

/* auxiliaries/flux_aux_vapor.F90:20-70 */
static inline double qsur_cclm(double fice, double ps, double ts) {
  const double aw = 17.2693882, ai = 21.8745584, t1 = 273.16, t2w = 35.86, t2i = 7.66,
               p0 = 610.78;
  double alpha = aw + (ai - aw) * fice;
  double t2 = t2w + (t2i - t2w) * fice;
  double e = p0 * exp(alpha * (ts - t1) / (ts - t2));
  return (R_D / R_V) * e / (ps - (1.0 - R_D / R_V) * e);
}

/* mass/flux_mass_evap.F90:22-85 (MOM5 == CCLM with another coefficient, :87-115) */
static inline double meva_cclm(double a, double ps, double qa, double qs, double ts,
                               double u, double v) {
  double tt = ts * (1.0 + (R_V / R_D - 1.0) * qs);
  double vel = sqrt(u * u + v * v);
  double fa = a * fmax(vel, U_MIN) * ps / (R_D * tt);
  return fa * (qs - qa);
}

/* mass/flux_mass_evap.F90:117-158 */
static inline double meva_rco(double qa, double ts, double u, double v) {
  const double rho_a = 1.225, c_aw = 1.15E-03, eps = 0.62197, p_0 = 1.013E+05,
               r = 6.1078E+02, c_1 = 17.269, c_2 = 35.86;
  double e_w = r * exp(c_1 * (ts - 273.15) / (ts - c_2));
  double q_w = eps * e_w / p_0;
  double vel = sqrt(u * u + v * v);
  return rho_a * c_aw * vel * (q_w - qa);
}

/* heat/flux_heat_sensible.F90:24-95 */
static inline double hsen_cclm(double a, double pa, double ps, double qs, double ta,
                               double ts, double u, double v) {
  double tt = ts * (1.0 + (R_V / R_D - 1.0) * qs);
  double vel = sqrt(u * u + v * v);
  double fa = a * fmax(vel, U_MIN) * ps / (R_D * tt);
  double ef = pow(ps / pa, R_D / C_P);
  return fa * C_P * (ts - ta * ef);
}

/* heat/flux_heat_sensible.F90:136-165 */
static inline double hsen_rco(double ta, double ts, double u, double v) {
  const double rho_a = 1.225, c_pa = 1.008E+03;
  double c_aw = (ta < ts) ? 1.13E-03 : 0.66E-03;
  double vel = sqrt(u * u + v * v);
  return rho_a * c_pa * c_aw * vel * (ts - ta);
}

/* momentum/flux_momentum.F90:22-71 */
static inline void mom_cclm(double a, double ps, double qs, double ts, double u, double v,
                            double *east, double *north) {
  double tt = ts * (1.0 + (R_V / R_D - 1.0) * qs);
  double vel = sqrt(u * u + v * v);
  double fa = a * vel * ps / (R_D * tt);
  *east = -(fa * u);
  *north = -(fa * v);
}

/* momentum/flux_momentum.F90:107-136 */
static inline void mom_rco(double u, double v, double *east, double *north) {
  const double rho_a = 1.225;
  double vel = sqrt(u * u + v * v);
  double c_aw = (vel < 11.0) ? 1.2E-03 : 0.49E-03 + 0.065E-03 * vel;
  *east = -(rho_a * c_aw * vel * u);
  *north = -(rho_a * c_aw * vel * v);
}

/* radiation/flux_radiation_blackbody.F90:22-42; T**4 is lowered by flang as
 * ((T*T)*T)*T (checked in the compiled reference object). */
static inline double rbbr_stbo(double ts) { return SIGMA * (ts * ts * ts * ts); }

/* ---------------- calc_* loops (flux_calculator_calculate.F90) ---------------- */

#define F(s, g, v) (st->field[(s)][(g)-1][(v)])
#define METHOD(f, s) (st->method[(f)][(s)-1])

static void zero_range(double *x, int j0, int j1) {
  for (int j = j0; j < j1; ++j) x[j] = 0.0;
}

/* calc:25-50 */
static void svs_range(fco_state *st, int g, int j0, int j1) {
  int flux = FCO_F_QSUR_T + (g - 1);
  for (int i = 1; i <= st->num_surface_types; ++i) {
    if (METHOD(flux, i) != FCO_M_CCLM) continue; /* 'none'/'copy': nothing computed */
    double *q = F(i, g, FCO_QSUR);
    const double *fi = F(i, g, FCO_FICE), *ps = F(i, g, FCO_PSUR), *ts = F(i, g, FCO_TSUR);
    for (int j = j0; j < j1; ++j) q[j] = qsur_cclm(fi[j], ps[j], ts[j]);
  }
}

/* calc:54-120 (P2: TATM is bound to the temperature_surface slot) */
static void meva_range(fco_state *st, int j0, int j1) {
  for (int i = 1; i <= st->num_surface_types; ++i) {
    int m = METHOD(FCO_F_MEVA, i);
    if (m == FCO_M_NONE) continue;
    double *out = F(i, 1, FCO_MEVA);
    if (m == FCO_M_ZERO) {
      zero_range(out, j0, j1);
    } else if (m == FCO_M_CCLM || m == FCO_M_MOM5) {
      const double *a = F(i, 1, m == FCO_M_CCLM ? FCO_AMOI : FCO_CMOI);
      const double *ps = F(i, 1, FCO_PSUR), *qa = F(i, 1, FCO_QATM), *qs = F(i, 1, FCO_QSUR),
                   *ta = F(i, 1, FCO_TATM), *u = F(i, 1, FCO_UATM), *v = F(i, 1, FCO_VATM);
      for (int j = j0; j < j1; ++j) out[j] = meva_cclm(a[j], ps[j], qa[j], qs[j], ta[j], u[j], v[j]);
    } else if (m == FCO_M_RCO) {
      const double *qa = F(i, 1, FCO_QATM), *ts = F(i, 1, FCO_TSUR), *u = F(i, 1, FCO_UATM),
                   *v = F(i, 1, FCO_VATM);
      for (int j = j0; j < j1; ++j) out[j] = meva_rco(qa[j], ts[j], u[j], v[j]);
    }
    /* calc:112-116: bias added for every method != none, also 'copy' (aliased array) */
    if (st->lcorrections) {
      const double *c = st->corrections + (st->current_month - 1);
      for (int j = j0; j < j1; ++j) out[j] = out[j] + c[(size_t)j * 12];
    }
  }
}

/* calc:124-154 */
static void hlat_range(fco_state *st, int j0, int j1) {
  for (int i = 1; i <= st->num_surface_types; ++i) {
    int m = METHOD(FCO_F_HLAT, i);
    if (m == FCO_M_NONE) continue;
    double *out = F(i, 1, FCO_HLAT);
    if (m == FCO_M_ZERO) {
      zero_range(out, j0, j1);
    } else if (m == FCO_M_WATER || m == FCO_M_ICE) {
      const double L = (m == FCO_M_WATER) ? L_V : L_S;
      const double *e = F(i, 1, FCO_MEVA);
      for (int j = j0; j < j1; ++j) out[j] = e[j] * L;
    }
  }
}

/* calc:156-208 (P3: QATM is bound to the specific_vapor_content_surface slot) */
static void hsen_range(fco_state *st, int j0, int j1) {
  for (int i = 1; i <= st->num_surface_types; ++i) {
    int m = METHOD(FCO_F_HSEN, i);
    if (m == FCO_M_NONE) continue;
    double *out = F(i, 1, FCO_HSEN);
    const double *ta = F(i, 1, FCO_TATM), *ts = F(i, 1, FCO_TSUR), *u = F(i, 1, FCO_UATM),
                 *v = F(i, 1, FCO_VATM);
    if (m == FCO_M_ZERO) {
      zero_range(out, j0, j1);
    } else if (m == FCO_M_CCLM || m == FCO_M_MOM5) {
      const double *a = F(i, 1, m == FCO_M_CCLM ? FCO_AMOI : FCO_CHEA);
      const double *pa = F(i, 1, FCO_PATM), *ps = F(i, 1, FCO_PSUR), *qa = F(i, 1, FCO_QATM);
      for (int j = j0; j < j1; ++j)
        out[j] = hsen_cclm(a[j], pa[j], ps[j], qa[j], ta[j], ts[j], u[j], v[j]);
    } else if (m == FCO_M_RCO) {
      for (int j = j0; j < j1; ++j) out[j] = hsen_rco(ta[j], ts[j], u[j], v[j]);
    }
  }
}

/* calc:212-316 (east: keep component 1, north: keep component 2) */
static void mom_range(fco_state *st, int g, int north, int j0, int j1) {
  int var = north ? FCO_VMOM : FCO_UMOM;
  for (int i = 1; i <= st->num_surface_types; ++i) {
    int m = METHOD(FCO_F_MOM, i);
    if (m == FCO_M_NONE) continue;
    double *out = F(i, g, var);
    const double *u = F(i, g, FCO_UATM), *v = F(i, g, FCO_VATM);
    double e, n;
    if (m == FCO_M_ZERO) {
      zero_range(out, j0, j1);
    } else if (m == FCO_M_CCLM || m == FCO_M_MOM5) {
      const double *a = F(i, g, m == FCO_M_CCLM ? FCO_AMOM : FCO_CMOM);
      const double *ps = F(i, g, FCO_PSUR), *qs = F(i, g, FCO_QSUR), *ts = F(i, g, FCO_TSUR);
      for (int j = j0; j < j1; ++j) {
        mom_cclm(a[j], ps[j], qs[j], ts[j], u[j], v[j], &e, &n);
        out[j] = north ? n : e;
      }
    } else if (m == FCO_M_RCO) {
      for (int j = j0; j < j1; ++j) {
        mom_rco(u[j], v[j], &e, &n);
        out[j] = north ? n : e;
      }
    }
  }
}

/* calc:320-345 */
static void rbbr_range(fco_state *st, int j0, int j1) {
  for (int i = 1; i <= st->num_surface_types; ++i) {
    int m = METHOD(FCO_F_RBBR, i);
    if (m == FCO_M_NONE) continue;
    double *out = F(i, 1, FCO_RBBR);
    if (m == FCO_M_ZERO) {
      zero_range(out, j0, j1);
    } else if (m == FCO_M_STBO) {
      const double *ts = F(i, 1, FCO_TSUR);
      for (int j = j0; j < j1; ++j) out[j] = rbbr_stbo(ts[j]);
    }
  }
}

/* calc:347-364 (P6: the reference dereferences unconditionally; we skip when unbound) */
static int rsdr_range(fco_state *st, int j0, int j1) {
  const double *rsdd = F(0, 1, FCO_RSDD);
  if (!rsdd) return 0;
  for (int i = 1; i <= st->num_surface_types; ++i) {
    double *out = F(i, 1, FCO_RSDR);
    if (!out) return 0;
    for (int j = j0; j < j1; ++j) out[j] = rsdd[j];
  }
  return 1;
}

/* calc:368-385 (P7: only when the type-0 array is allocated, summed in order i=1..T) */
static void avg_range(fco_state *st, int g, int var, int j0, int j1) {
  if (!st->allocated[0][g - 1][var]) return;
  double *x0 = F(0, g, var);
  zero_range(x0, j0, j1);
  for (int i = 1; i <= st->num_surface_types; ++i) {
    const double *x = F(i, g, var), *fa = F(i, g, FCO_FARE);
    for (int j = j0; j < j1; ++j) x0[j] = x0[j] + x[j] * fa[j];
  }
}

/* ---------------- public API ---------------- */

void fco_calc_spec_vapor_surface(fco_state *st, int g) { svs_range(st, g, 0, st->grid_size[g - 1]); }
void fco_calc_flux_mass_evap(fco_state *st) { meva_range(st, 0, st->grid_size[0]); }
void fco_calc_flux_heat_latent(fco_state *st) { hlat_range(st, 0, st->grid_size[0]); }
void fco_calc_flux_heat_sensible(fco_state *st) { hsen_range(st, 0, st->grid_size[0]); }
void fco_calc_flux_momentum_east(fco_state *st, int g) { mom_range(st, g, 0, 0, st->grid_size[g - 1]); }
void fco_calc_flux_momentum_north(fco_state *st, int g) { mom_range(st, g, 1, 0, st->grid_size[g - 1]); }
void fco_calc_flux_radiation_blackbody(fco_state *st) { rbbr_range(st, 0, st->grid_size[0]); }
int fco_distribute_shortwave_radiation_flux(fco_state *st) { return rsdr_range(st, 0, st->grid_size[0]); }
void fco_average_across_surface_types(fco_state *st, int g, int var) {
  avg_range(st, g, var, 0, st->grid_size[g - 1]);
}

/* basic:463-522: dst zeroed, then sequential COO scatter-add in link order */
void fco_do_regridding(fco_state *st, int var, int surface_type) {
  static const int from_g[4] = {2, 3, 1, 1}, to_g[4] = {1, 1, 2, 3}, bit[4] = {1, 1, 2, 4};
  for (int s = 1; s <= FCO_MAX_SURFACE_TYPES; ++s) {
    if (!(s == surface_type || surface_type == 0)) continue;
    for (int k = 0; k < 4; ++k) {
      if (!(st->put_to[s][from_g[k] - 1][var] & bit[k])) continue;
      const fco_matrix *mx = &st->regrid[k];
      double *dst = F(s, to_g[k], var);
      const double *src = F(s, from_g[k], var);
      zero_range(dst, 0, st->grid_size[to_g[k] - 1]);
      for (int e = 0; e < mx->num_elements; ++e)
        dst[mx->dst_index[e] - 1] = dst[mx->dst_index[e] - 1] + src[mx->src_index[e] - 1] * mx->weight[e];
    }
  }
}

/* datetime_helpers.py:4-13: datetime.strptime(str(init_date), "%Y%m%d") + timedelta(seconds) */
static int64_t days_from_civil(int64_t y, int m, int d) {
  y -= m <= 2;
  int64_t era = (y >= 0 ? y : y - 399) / 400;
  int64_t yoe = y - era * 400;
  int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}
int fco_current_month(int32_t init_date, int64_t seconds) {
  int64_t y = init_date / 10000;
  int m = (init_date / 100) % 100, d = init_date % 100;
  int64_t days = days_from_civil(y, m, d);
  int64_t q = seconds / 86400;
  if (seconds % 86400 != 0 && seconds < 0) q -= 1; /* floor */
  int64_t z = days + q + 719468;
  int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  int64_t doe = z - era * 146097;
  int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  int64_t mp = (5 * doy + 2) / 153;
  return (int)(mp < 10 ? mp + 3 : mp - 9);
}

/* One coupling step in the order of flux_calculator.F90:902-991 (no regridding; the
 * type-0 averages are the caller's, as in the reference put loop). */
static void step_range(fco_state *st, int j0t, int j1t, int j0u, int j1u, int j0v, int j1v) {
  rbbr_range(st, j0t, j1t);
  svs_range(st, 1, j0t, j1t);
  svs_range(st, 2, j0u, j1u);
  svs_range(st, 3, j0v, j1v);
  meva_range(st, j0t, j1t);
  hlat_range(st, j0t, j1t);
  hsen_range(st, j0t, j1t);
  mom_range(st, 2, 0, j0u, j1u);
  mom_range(st, 3, 1, j0v, j1v);
  rsdr_range(st, j0t, j1t);
}

void fco_step(fco_state *st) {
  step_range(st, 0, st->grid_size[0], 0, st->grid_size[1], 0, st->grid_size[2]);
}

int fco_step_threads(fco_state *st, int nthreads) {
#ifdef _OPENMP
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    int t = omp_get_thread_num(), p = omp_get_num_threads();
    int r[3][2];
    for (int g = 0; g < 3; ++g) { /* APPLE ranges: decomp_def.F90:23-31 */
      int n = st->grid_size[g], part = n / p;
      r[g][0] = t * part;
      r[g][1] = (t < p - 1) ? (t + 1) * part : n;
    }
    step_range(st, r[0][0], r[0][1], r[1][0], r[1][1], r[2][0], r[2][1]);
  }
  return 0;
#else
  (void)nthreads;
  fco_step(st);
  return 0;
#endif
}

void fco_remap_apply(int64_t n_links, const int32_t *src, const int32_t *dst, const double *w,
                     const double *x, int64_t n_dst, double *out) {
  for (int64_t d = 0; d < n_dst; ++d) out[d] = 0.0;
  for (int64_t k = 0; k < n_links; ++k) out[dst[k]] = out[dst[k]] + w[k] * x[src[k]];
}

void fco_atmos_accumulate(int64_t n_cells, const int32_t *atmos_index, const double *weight,
                          const double *x_field, int64_t n_atmos, double *out) {
  for (int64_t a = 0; a < n_atmos; ++a) out[a] = 0.0;
  for (int64_t x = 0; x < n_cells; ++x) {
    const int64_t a = atmos_index[x];
    out[a] = out[a] + weight[x] * x_field[x];
  }
}
