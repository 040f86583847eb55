/*
 * fco.h -- CPU ORACLE for the exchange-grid flux path.  TEST INFRASTRUCTURE ONLY.
 *
 * Nothing in the product (components.flux_calculator_amd/, include/) links, loads or
 * calls this code.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg use it, and only as the checker / the timed CPU baseline.
 *
 * The state struct mirrors the reference data model one-to-one:
 *   local_field(0:MAX_SURFACE_TYPES, 3)%var(MAX_VARNAMES)%field(:)
 *   (flux_calculator_basic.F90:86-103, flux_calculator.F90:159)
 * Every (surface_type, grid, var) slot holds a raw pointer; NULL == not ASSOCIATED.
 * Aliases (atmosphere fields distributed to all surface types, 'copy' methods,
 * -2e20 namelist values, uniform type-0 outputs) are expressed, exactly as in the
 * reference, by storing the SAME pointer in several slots.
 *
 * The identical struct is consumed by oracle/ref_harness.F90 (bind(C) derived type),
 * which drives the reference flux_lib compiled from /root/reference sources.
 */
#ifndef FCO_H
#define FCO_H
#include <stdint.h>

#define FCO_MAX_SURFACE_TYPES 10 /* flux_calculator_basic.F90:28 */
#define FCO_NUM_VARS 35          /* flux_calculator_basic.F90:42 */
#define FCO_NUM_FLUXES 8

/* 0-based var ids = reference idx_* - 1 (flux_calculator_basic.F90:43-51) */
enum {
  FCO_ALBE, FCO_ALBA, FCO_AMOI, FCO_AMOM, FCO_FARE, FCO_FICE, FCO_PATM, FCO_PSUR,
  FCO_QATM, FCO_TATM, FCO_TSUR, FCO_UATM, FCO_VATM, FCO_U10M, FCO_V10M,
  FCO_CMOM, FCO_CMOI, FCO_CHEA, FCO_QSUR, FCO_HLAT, FCO_HSEN,
  FCO_MEVA, FCO_MPRE, FCO_MRAI, FCO_MSNO,
  FCO_RBBR, FCO_RLWD, FCO_RLWU, FCO_RSID, FCO_RSIU, FCO_RSIN, FCO_RSDD, FCO_RSDR,
  FCO_UMOM, FCO_VMOM
};

/* method strings of the namelist which_* tables (flux_calculator.F90:99-107) */
enum { FCO_M_NONE = 0, FCO_M_ZERO, FCO_M_COPY, FCO_M_CCLM, FCO_M_MOM5, FCO_M_RCO,
       FCO_M_WATER, FCO_M_ICE, FCO_M_STBO };

/* which_* tables: spec_vapor_surface_{t,u,v}, mass_evap, heat_latent, heat_sensible,
 * momentum, radiation_blackbody */
enum { FCO_F_QSUR_T = 0, FCO_F_QSUR_U, FCO_F_QSUR_V, FCO_F_MEVA, FCO_F_HLAT, FCO_F_HSEN,
       FCO_F_MOM, FCO_F_RBBR };

/* regridding matrices, flux_calculator.F90:330-337 order */
enum { FCO_RG_U_TO_T = 0, FCO_RG_V_TO_T, FCO_RG_T_TO_U, FCO_RG_T_TO_V };

typedef struct {
  int32_t num_elements;      /* basic:118 */
  int32_t pad;
  const int32_t *src_index;  /* 1-based, offset-corrected (io:183-191) */
  const int32_t *dst_index;
  const double *weight;
} fco_matrix;

typedef struct {
  int32_t num_surface_types;
  int32_t grid_size[3];
  int32_t method[FCO_NUM_FLUXES][FCO_MAX_SURFACE_TYPES]; /* [flux][type-1] */
  int32_t lcorrections;      /* bias_corrections.F90:32 */
  int32_t current_month;     /* 1..12, from datetime_helpers.get_current_date */
  const double *corrections; /* Fortran corrections(1,12,grid_size(1)): [cell][month] */
  double *field[FCO_MAX_SURFACE_TYPES + 1][3][FCO_NUM_VARS];
  uint8_t allocated[FCO_MAX_SURFACE_TYPES + 1][3][FCO_NUM_VARS];
  uint8_t put_to[FCO_MAX_SURFACE_TYPES + 1][3][FCO_NUM_VARS]; /* bit0 t, bit1 u, bit2 v */
  fco_matrix regrid[4];
} fco_state;

#ifdef __cplusplus
extern "C" {
#endif
/* flux_calculator_calculate.F90 restated (calc:25-385) */
void fco_calc_spec_vapor_surface(fco_state *st, int which_grid);
void fco_calc_flux_mass_evap(fco_state *st);
void fco_calc_flux_heat_latent(fco_state *st);
void fco_calc_flux_heat_sensible(fco_state *st);
void fco_calc_flux_momentum_east(fco_state *st, int which_grid);
void fco_calc_flux_momentum_north(fco_state *st, int which_grid);
void fco_calc_flux_radiation_blackbody(fco_state *st);
int  fco_distribute_shortwave_radiation_flux(fco_state *st);
void fco_average_across_surface_types(fco_state *st, int which_grid, int var);
/* flux_calculator_basic.F90:463-522 restated */
void fco_do_regridding(fco_state *st, int var, int surface_type);
/* datetime_helpers.py:4-13 restated: month of init_date(YYYYMMDD) + seconds */
int  fco_current_month(int32_t init_date, int64_t seconds);
/* Exchange-grid -> atmosphere accumulation that OASIS3-MCT performs on oasis_put of the
 * type-0 fields ('S A xxxx 00', create_namcouple.F90:92-98, LOCTRANS MAPPING): SCRIP
 * weight application out[a] = sum_x w[x] * x_field[x] over the exchange cells x of atmosphere
 * cell a.  Not in the reference repository (OASIS is a sibling component): restated from the
 * published SCRIP remap, PARITY UNPINNED.  Cells are summed in increasing x, from 0.0. */
/* OASIS-style SCRIP weight application of a remapping file to a target (model) grid:
 * out[d] = 0 for all d, then out[dst[k]] += w[k] * x[src[k]] for k in link order
 * (0-based indices).  OASIS3-MCT itself is not in the reference: parity unpinned. */
void fco_remap_apply(int64_t n_links, const int32_t *src, const int32_t *dst, const double *w,
                     const double *x, int64_t n_dst, double *out);
void fco_atmos_accumulate(int64_t n_cells, const int32_t *atmos_index, const double *weight,
                          const double *x_field, int64_t n_atmos, double *out);
/* one full coupling step in reference order (flux_calculator.F90:902-991), no regridding */
void fco_step(fco_state *st);
/* multi-threaded (OpenMP) variant of fco_step over contiguous cell ranges: the reference's
 * MPI range decomposition on the host cores; T=1 hot path only (returns -1 otherwise) */
int  fco_step_threads(fco_state *st, int nthreads);
#ifdef __cplusplus
}
#endif
#endif
