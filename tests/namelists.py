"""flux_calculator.nml texts for the set-up / namcouple / driver tests.

Written here from the namelist variables the reference declares (flux_calculator.F90:55-129);
the IOW-ESM example set-ups themselves are not in the reference repository.
"""
import numpy as np


def regrid_matrices(grids, seed=11):
    """Random rank-local COO links (1-based) for the four regriddings (FCX_U_TO_T,
    FCX_V_TO_T, FCX_T_TO_U, FCX_T_TO_V): 1-3 links per destination cell, weights a convex
    combination (an interpolation), links shuffled."""
    rng = np.random.default_rng(seed)
    nt, nu, nv = grids
    mats = {}
    for which, (ns, nd) in {0: (nu, nt), 1: (nv, nt), 2: (nt, nu), 3: (nt, nv)}.items():
        per = rng.integers(1, 4, nd)
        dst = np.repeat(np.arange(1, nd + 1), per)
        order = rng.permutation(dst.size)
        w = rng.uniform(0.1, 1.0, dst.size)
        w /= np.bincount(dst - 1, weights=w)[dst - 1]
        mats[which] = (rng.integers(1, ns + 1, dst.size), dst[order], w[order])
    return {"matrices": mats}


# MOM5_Baltic under CCLM_Eurocordex: surface type 1 = open water, 2 = sea ice.  Every field
# is received on the t grid; what the momentum fluxes need on the u and v grids is
# regridded there after reading (prepare_regridding of the received fields).
MOM5_BALTIC = """
! flux_calculator.nml for the tests
&input
  timestep      = 600
  num_timesteps = 3
  name_atmos_model       = 'CCLM_Eurocordex'
  name_bottom_model(1)   = 'MOM5_Baltic'
  letter_bottom_model(1) = 'M'
  num_tasks_per_model(1) = 1

  name_bottom_var_t(1,1,:) = 'TSUR', 'FARE', 'FICE', 'ALBE', 'CMOI', 'CHEA', 'CMOM'
  name_bottom_var_t(1,2,:) = 'TSUR', 'FARE', 'FICE', 'ALBE', 'CMOI', 'CHEA', 'CMOM'
  val_bottom_var_t(1,2,3)  = 1.0            ! ice type: FICE = 1 everywhere
  val_bottom_var_t(1,2,7)  = -2.0e20        ! ice CMOM: the water type's array
  name_atmos_var_t = 'PATM', 'PSUR', 'QATM', 'TATM', 'UATM', 'VATM'
  regrid_t_to_u(1,1,:) = 'TSUR', 'FICE', 'CMOM', 'PSUR', 'TATM', 'UATM', 'VATM'
  regrid_t_to_v(1,1,:) = 'TSUR', 'FICE', 'CMOM', 'PSUR', 'TATM', 'UATM', 'VATM'

  which_spec_vapor_surface_t(1,1:2) = 'CCLM', 'CCLM'
  which_spec_vapor_surface_u(1,1)   = 'CCLM'
  which_spec_vapor_surface_v(1,1)   = 'CCLM'
  which_flux_mass_evap(1,1:2)           = 'MOM5', 'MOM5'
  which_flux_heat_latent(1,1:2)         = 'water', 'ice'
  which_flux_heat_sensible(1,1:2)       = 'MOM5', 'MOM5'
  which_flux_momentum(1,1:2)            = 'MOM5', 'copy'
  which_flux_radiation_blackbody(1,1:2) = 'StBo', 'StBo'

  name_send_t = 'MEVA', 'HLAT', 'HSEN', 'RBBR', 'TSUR', 'RLWU'
  send_uniform_t(1,4) = .true.              ! RBBR: one field for all types
  send_to_bottom_t(1,5) = F                 ! TSUR goes to the atmosphere only
  val_flux_t(6) = -5.0                      ! RLWU is not computed: default value
  name_send_u = 'UMOM'
  name_send_v = 'VMOM'
  send_uniform_u(1,1) = T                   ! no FARE on u / v: momentum is sent uniform
  send_uniform_v(1,1) = T
/
&correctionsctl
  init_date = 20000101
  lcorrections = .true.
/
"""

# CCLM-type single surface type, the second of two bottom models (rank 1): everything is
# received on the t grid and regridded t -> u / t -> v after reading; UMOM u -> t and
# VMOM v -> t after the calculation, sent from the t grid.
CCLM_REGRID = """
&input
  timestep = 3600, num_timesteps = 2
  verbosity_level = 2
  name_atmos_model = 'CCLM_Eurocordex'
  name_bottom_model = 'RCO_Baltic', 'MOM5_Baltic'
  letter_bottom_model = 'R', 'M'
  num_tasks_per_model = 1, 1
  name_bottom_var_t(2,1,:) = 'TSUR', 'FICE', 'FARE'
  name_atmos_var_t = 'PATM', 'PSUR', 'QATM', 'TATM', 'UATM', 'VATM', 'AMOI', 'AMOM'
  regrid_t_to_u(2,1,:) = 'TSUR', 'FICE', 'PSUR', 'QATM', 'TATM', 'UATM', 'VATM', 'AMOM'
  regrid_t_to_v(2,1,:) = 'TSUR', 'FICE', 'PSUR', 'QATM', 'TATM', 'UATM', 'VATM', 'AMOM'
  regrid_u_to_t(2,1,1) = 'UMOM'
  regrid_v_to_t(2,1,1) = 'VMOM'
  which_spec_vapor_surface_t(2,1) = 'CCLM'
  which_spec_vapor_surface_u(2,1) = 'CCLM'
  which_spec_vapor_surface_v(2,1) = 'CCLM'
  which_flux_mass_evap(2,1) = 'CCLM'
  which_flux_heat_latent(2,1) = 'water'
  which_flux_heat_sensible(2,1) = 'CCLM'
  which_flux_momentum(2,1) = 'CCLM'
  which_flux_radiation_blackbody(2,1) = 'StBo'
  name_send_t = 'MEVA', 'HLAT', 'HSEN', 'RBBR', 'UMOM', 'VMOM'
  send_uniform_t(2,1:6) = 6*.true.          ! one surface type: one field per flux
/
"""
