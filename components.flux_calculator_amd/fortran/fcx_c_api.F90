! fcx_c_api.F90 -- iso_c_binding interfaces of include/fcx.h for Fortran hosts.
!
! One interface per C entry point, plain C types only (integers, doubles, c_ptr).  Every
! function returns the C status (FCX_OK == 0); fcx_error_message() turns fcx_last_error()
! into a Fortran string.
MODULE fcx_c_api
  USE, INTRINSIC :: iso_c_binding
  IMPLICIT NONE

  INTEGER(c_int), PARAMETER :: FCX_OK = 0
  INTEGER(c_int), PARAMETER :: FCX_PHASE_EARLY = 1, FCX_PHASE_NORMAL = 2, FCX_PHASE_ALL = 3
  INTEGER(c_int), PARAMETER :: FCX_MEM_HOST = 0, FCX_MEM_DEVICE = 1, FCX_ALLOCATED = 2
  INTEGER(c_int), PARAMETER :: FCX_CORR_CELL_MAJOR = 0, FCX_CORR_MONTH_MAJOR = 1
  INTEGER(c_int), PARAMETER :: FCX_PRECISION_F64 = 0, FCX_PRECISION_F32 = 1
  ! which_* tables (enum fcx_flux)
  INTEGER(c_int), PARAMETER :: FCX_SPEC_VAPOR_SURFACE_T = 0, FCX_SPEC_VAPOR_SURFACE_U = 1, &
                               FCX_SPEC_VAPOR_SURFACE_V = 2, FCX_FLUX_MASS_EVAP = 3, &
                               FCX_FLUX_HEAT_LATENT = 4, FCX_FLUX_HEAT_SENSIBLE = 5, &
                               FCX_FLUX_MOMENTUM = 6, FCX_FLUX_RADIATION_BLACKBODY = 7
  ! regridding matrices (enum fcx_regrid)
  INTEGER(c_int), PARAMETER :: FCX_U_TO_T = 0, FCX_V_TO_T = 1, FCX_T_TO_U = 2, FCX_T_TO_V = 3
  ! fcx_set_option (enum fcx_option)
  INTEGER(c_int), PARAMETER :: FCX_OPT_NONTEMPORAL = 3, FCX_OPT_ATMOS_IN_RUN = 5, &
                               FCX_OPT_PIPELINE_CHUNKS = 7, FCX_OPT_ZERO_COPY = 9, FCX_OPT_TIMING = 10, &
                               FCX_OPT_TILED_LAYOUT = 11, FCX_OPT_REMAP_PACK = 13, &
                               FCX_OPT_HOST_STAGING = 15, FCX_OPT_HOST_THREADS = 16, &
                               FCX_OPT_ATMOS_HALO = 17, FCX_OPT_DEFERRED_SCATTER = 18, &
                               FCX_OPT_LIB_SPANS = 19
  ! retired in version 3: accepted by fcx_set_option and ignored
  INTEGER(c_int), PARAMETER :: FCX_OPT_PIN_HOST = 6, FCX_OPT_CARRY_HANDOFF = 14
  ! the RCCL unique id travels between the ranks as these many bytes (MPI_Bcast)
  INTEGER, PARAMETER :: FCX_COMM_ID_BYTES = 128

  INTERFACE
    FUNCTION fcx_last_error() BIND(C, name='fcx_last_error')
      IMPORT :: c_ptr
      TYPE(c_ptr) :: fcx_last_error
    END FUNCTION
    FUNCTION fcx_version() BIND(C, name='fcx_version')
      IMPORT :: c_int
      INTEGER(c_int) :: fcx_version
    END FUNCTION
    FUNCTION fcx_method_from_string(s, len) BIND(C, name='fcx_method_from_string')
      IMPORT :: c_int, c_char, c_size_t
      CHARACTER(kind=c_char), DIMENSION(*), INTENT(IN) :: s
      INTEGER(c_size_t), VALUE :: len
      INTEGER(c_int) :: fcx_method_from_string
    END FUNCTION
    FUNCTION fcx_current_month(init_date, seconds, month) BIND(C, name='fcx_current_month')
      IMPORT :: c_int, c_int32_t, c_int64_t
      INTEGER(c_int32_t), VALUE :: init_date
      INTEGER(c_int64_t), VALUE :: seconds
      INTEGER(c_int32_t), INTENT(OUT) :: month
      INTEGER(c_int) :: fcx_current_month
    END FUNCTION
    FUNCTION fcx_create(device, num_surface_types, grid_size, engine) BIND(C, name='fcx_create')
      IMPORT :: c_int, c_int32_t, c_ptr
      INTEGER(c_int), VALUE :: device, num_surface_types
      INTEGER(c_int32_t), DIMENSION(3), INTENT(IN) :: grid_size
      TYPE(c_ptr), INTENT(OUT) :: engine
      INTEGER(c_int) :: fcx_create
    END FUNCTION
    FUNCTION fcx_destroy(engine) BIND(C, name='fcx_destroy')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int) :: fcx_destroy
    END FUNCTION
    FUNCTION fcx_set_method(engine, flux, surface_type, method) BIND(C, name='fcx_set_method')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: flux, surface_type, method
      INTEGER(c_int) :: fcx_set_method
    END FUNCTION
    FUNCTION fcx_bind_field(engine, surface_type, grid, var, ptr, n, flags) BIND(C, name='fcx_bind_field')
      IMPORT :: c_int, c_ptr, c_int64_t
      TYPE(c_ptr), VALUE :: engine, ptr
      INTEGER(c_int), VALUE :: surface_type, grid, var, flags
      INTEGER(c_int64_t), VALUE :: n
      INTEGER(c_int) :: fcx_bind_field
    END FUNCTION
    FUNCTION fcx_set_corrections(engine, enabled, init_date, corr, n, layout) BIND(C, name='fcx_set_corrections')
      IMPORT :: c_int, c_int32_t, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine, corr
      INTEGER(c_int), VALUE :: enabled, layout
      INTEGER(c_int32_t), VALUE :: init_date
      INTEGER(c_int64_t), VALUE :: n
      INTEGER(c_int) :: fcx_set_corrections
    END FUNCTION
    FUNCTION fcx_set_regrid_matrix(engine, which, nnz, src, dst, w) BIND(C, name='fcx_set_regrid_matrix')
      IMPORT :: c_int, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine, src, dst, w
      INTEGER(c_int), VALUE :: which
      INTEGER(c_int64_t), VALUE :: nnz
      INTEGER(c_int) :: fcx_set_regrid_matrix
    END FUNCTION
    FUNCTION fcx_set_put_to(engine, surface_type, grid, var, mask) BIND(C, name='fcx_set_put_to')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: surface_type, grid, var, mask
      INTEGER(c_int) :: fcx_set_put_to
    END FUNCTION
    FUNCTION fcx_add_average(engine, phase, grid, var) BIND(C, name='fcx_add_average')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: phase, grid, var
      INTEGER(c_int) :: fcx_add_average
    END FUNCTION
    FUNCTION fcx_set_precision(engine, precision) BIND(C, name='fcx_set_precision')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: precision
      INTEGER(c_int) :: fcx_set_precision
    END FUNCTION
    FUNCTION fcx_commit(engine) BIND(C, name='fcx_commit')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int) :: fcx_commit
    END FUNCTION
    FUNCTION fcx_step(engine, phase, t) BIND(C, name='fcx_step')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: phase
      INTEGER(c_int32_t), VALUE :: t
      INTEGER(c_int) :: fcx_step
    END FUNCTION
    ! fcx_step without its final wait: outputs in the host arrays after fcx_synchronize
    FUNCTION fcx_step_async(engine, phase, t) BIND(C, name='fcx_step_async')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: phase
      INTEGER(c_int32_t), VALUE :: t
      INTEGER(c_int) :: fcx_step_async
    END FUNCTION
    ! one input field handed over after its oasis_get (staged by the engine's upload thread)
    FUNCTION fcx_upload_field(engine, surface_type, grid, var) BIND(C, name='fcx_upload_field')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: surface_type, grid, var
      INTEGER(c_int) :: fcx_upload_field
    END FUNCTION
    FUNCTION fcx_run(engine, phase, t) BIND(C, name='fcx_run')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: phase
      INTEGER(c_int32_t), VALUE :: t
      INTEGER(c_int) :: fcx_run
    END FUNCTION
    ! several engines' fcx_run, their fused flux passes as one launch (engines: c_ptr array)
    FUNCTION fcx_run_group(engines, n, phase, t) BIND(C, name='fcx_run_group')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), DIMENSION(*), INTENT(IN) :: engines
      INTEGER(c_int), VALUE :: n, phase
      INTEGER(c_int32_t), VALUE :: t
      INTEGER(c_int) :: fcx_run_group
    END FUNCTION
    FUNCTION fcx_upload(engine, phase) BIND(C, name='fcx_upload')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: phase
      INTEGER(c_int) :: fcx_upload
    END FUNCTION
    FUNCTION fcx_download(engine, phase) BIND(C, name='fcx_download')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: phase
      INTEGER(c_int) :: fcx_download
    END FUNCTION
    FUNCTION fcx_synchronize(engine) BIND(C, name='fcx_synchronize')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int) :: fcx_synchronize
    END FUNCTION
    FUNCTION fcx_calc_spec_vapor_surface(engine, which_grid) BIND(C, name='fcx_calc_spec_vapor_surface')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: which_grid
      INTEGER(c_int) :: fcx_calc_spec_vapor_surface
    END FUNCTION
    FUNCTION fcx_calc_flux_mass_evap(engine, t) BIND(C, name='fcx_calc_flux_mass_evap')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int32_t), VALUE :: t
      INTEGER(c_int) :: fcx_calc_flux_mass_evap
    END FUNCTION
    FUNCTION fcx_calc_flux_heat_latent(engine) BIND(C, name='fcx_calc_flux_heat_latent')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int) :: fcx_calc_flux_heat_latent
    END FUNCTION
    FUNCTION fcx_calc_flux_heat_sensible(engine) BIND(C, name='fcx_calc_flux_heat_sensible')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int) :: fcx_calc_flux_heat_sensible
    END FUNCTION
    FUNCTION fcx_calc_flux_momentum_east(engine, which_grid) BIND(C, name='fcx_calc_flux_momentum_east')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: which_grid
      INTEGER(c_int) :: fcx_calc_flux_momentum_east
    END FUNCTION
    FUNCTION fcx_calc_flux_momentum_north(engine, which_grid) BIND(C, name='fcx_calc_flux_momentum_north')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: which_grid
      INTEGER(c_int) :: fcx_calc_flux_momentum_north
    END FUNCTION
    FUNCTION fcx_calc_flux_radiation_blackbody(engine) BIND(C, name='fcx_calc_flux_radiation_blackbody')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int) :: fcx_calc_flux_radiation_blackbody
    END FUNCTION
    FUNCTION fcx_distribute_shortwave_radiation_flux(engine) &
        BIND(C, name='fcx_distribute_shortwave_radiation_flux')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int) :: fcx_distribute_shortwave_radiation_flux
    END FUNCTION
    FUNCTION fcx_average_across_surface_types(engine, which_grid, var) &
        BIND(C, name='fcx_average_across_surface_types')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: which_grid, var
      INTEGER(c_int) :: fcx_average_across_surface_types
    END FUNCTION
    FUNCTION fcx_do_regridding(engine, var, surface_type) BIND(C, name='fcx_do_regridding')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: var, surface_type
      INTEGER(c_int) :: fcx_do_regridding
    END FUNCTION
    ! ---- exchange -> atmosphere accumulation and its one collective (SURVEY.md 8e)
    FUNCTION fcx_set_atmos_map(engine, n_atmos, atmos_index, weight) BIND(C, name='fcx_set_atmos_map')
      IMPORT :: c_int, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine, atmos_index, weight
      INTEGER(c_int64_t), VALUE :: n_atmos
      INTEGER(c_int) :: fcx_set_atmos_map
    END FUNCTION
    FUNCTION fcx_add_atmos_field(engine, phase, surface_type, grid, var, out, flags) &
        BIND(C, name='fcx_add_atmos_field')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine, out
      INTEGER(c_int), VALUE :: phase, surface_type, grid, var, flags
      INTEGER(c_int) :: fcx_add_atmos_field
    END FUNCTION
    FUNCTION fcx_set_atmos_boundaries(engine, n_boundaries, left, right) BIND(C, name='fcx_set_atmos_boundaries')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int32_t), VALUE :: n_boundaries, left, right
      INTEGER(c_int) :: fcx_set_atmos_boundaries
    END FUNCTION
    FUNCTION fcx_atmos_finish(engine) BIND(C, name='fcx_atmos_finish')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int) :: fcx_atmos_finish
    END FUNCTION
    FUNCTION fcx_run_atmos(engine, phase) BIND(C, name='fcx_run_atmos')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: phase
      INTEGER(c_int) :: fcx_run_atmos
    END FUNCTION
    FUNCTION fcx_comm_unique_id(id) BIND(C, name='fcx_comm_unique_id')
      IMPORT :: c_int, c_int8_t
      INTEGER(c_int8_t), DIMENSION(*), INTENT(OUT) :: id
      INTEGER(c_int) :: fcx_comm_unique_id
    END FUNCTION
    FUNCTION fcx_comm_create(device, nranks, rank, id, comm) BIND(C, name='fcx_comm_create')
      IMPORT :: c_int, c_int8_t, c_ptr
      INTEGER(c_int), VALUE :: device, nranks, rank
      INTEGER(c_int8_t), DIMENSION(*), INTENT(IN) :: id
      TYPE(c_ptr), INTENT(OUT) :: comm
      INTEGER(c_int) :: fcx_comm_create
    END FUNCTION
    FUNCTION fcx_comm_destroy(comm) BIND(C, name='fcx_comm_destroy')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: comm
      INTEGER(c_int) :: fcx_comm_destroy
    END FUNCTION
    FUNCTION fcx_set_comm(engine, comm) BIND(C, name='fcx_set_comm')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine, comm
      INTEGER(c_int) :: fcx_set_comm
    END FUNCTION
    FUNCTION fcx_set_option(engine, option, value) BIND(C, name='fcx_set_option')
      IMPORT :: c_int, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: option
      INTEGER(c_int64_t), VALUE :: value
      INTEGER(c_int) :: fcx_set_option
    END FUNCTION
    FUNCTION fcx_staging_bytes(engine, bytes) BIND(C, name='fcx_staging_bytes')
      IMPORT :: c_int, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int64_t), INTENT(OUT) :: bytes
      INTEGER(c_int) :: fcx_staging_bytes
    END FUNCTION
    FUNCTION fcx_zero_copy_bytes(engine, bytes) BIND(C, name='fcx_zero_copy_bytes')
      IMPORT :: c_int, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int64_t), INTENT(OUT) :: bytes
      INTEGER(c_int) :: fcx_zero_copy_bytes
    END FUNCTION
    ! retired in version 3 (always 0), kept for one release
    FUNCTION fcx_pinned_bytes(engine, bytes) BIND(C, name='fcx_pinned_bytes')
      IMPORT :: c_int, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int64_t), INTENT(OUT) :: bytes
      INTEGER(c_int) :: fcx_pinned_bytes
    END FUNCTION
    FUNCTION fcx_handoff_recoveries(engine, count) BIND(C, name='fcx_handoff_recoveries')
      IMPORT :: c_int, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int64_t), INTENT(OUT) :: count
      INTEGER(c_int) :: fcx_handoff_recoveries
    END FUNCTION
    ! ---- exchange -> model remaps (the OASIS 'S' maps to a bottom model, SURVEY.md 8f rank 3):
    ! src/dst 0-based cells, links in file order; outputs REAL(wp) arrays of n_dst cells
    FUNCTION fcx_add_remap(engine, n_dst, n_links, src_cell, dst_cell, weight, remap_id) &
        BIND(C, name='fcx_add_remap')
      IMPORT :: c_int, c_int32_t, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine, src_cell, dst_cell, weight
      INTEGER(c_int64_t), VALUE :: n_dst, n_links
      INTEGER(c_int32_t), INTENT(OUT) :: remap_id
      INTEGER(c_int) :: fcx_add_remap
    END FUNCTION
    FUNCTION fcx_add_remap_field(engine, remap_id, phase, surface_type, grid, var, out, flags) &
        BIND(C, name='fcx_add_remap_field')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), VALUE :: engine, out
      INTEGER(c_int32_t), VALUE :: remap_id
      INTEGER(c_int), VALUE :: phase, surface_type, grid, var, flags
      INTEGER(c_int) :: fcx_add_remap_field
    END FUNCTION
    FUNCTION fcx_remap_info(engine, remap_id, scatter, packed) BIND(C, name='fcx_remap_info')
      IMPORT :: c_int, c_int32_t, c_double, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int32_t), VALUE :: remap_id
      REAL(c_double), INTENT(OUT) :: scatter
      INTEGER(c_int32_t), INTENT(OUT) :: packed
      INTEGER(c_int) :: fcx_remap_info
    END FUNCTION
    ! ---- library-owned page-locked host memory (c_f_pointer it onto local_field arrays)
    FUNCTION fcx_host_malloc(bytes, ptr) BIND(C, name='fcx_host_malloc')
      IMPORT :: c_int, c_size_t, c_ptr
      INTEGER(c_size_t), VALUE :: bytes
      TYPE(c_ptr), INTENT(OUT) :: ptr
      INTEGER(c_int) :: fcx_host_malloc
    END FUNCTION
    FUNCTION fcx_host_free(ptr) BIND(C, name='fcx_host_free')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: ptr
      INTEGER(c_int) :: fcx_host_free
    END FUNCTION
    ! engines in the merged launch of the engine's last fcx_run_group (0: ran as fcx_run)
    FUNCTION fcx_last_group_size(engine, members) BIND(C, name='fcx_last_group_size')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int32_t), INTENT(OUT) :: members
      INTEGER(c_int) :: fcx_last_group_size
    END FUNCTION
    ! 1: the boundary-exchange signature agreement before every exchange (0: first of each)
    FUNCTION fcx_comm_verify(comm, every_exchange) BIND(C, name='fcx_comm_verify')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: comm
      INTEGER(c_int), VALUE :: every_exchange
      INTEGER(c_int) :: fcx_comm_verify
    END FUNCTION
    ! ---- the host's abort routine (oasis_abort, flux_calculator.F90:883-887): a BIND(C)
    ! subroutine taking CHARACTER(kind=c_char), DIMENSION(*) (NUL-terminated), registered
    ! with c_funloc; fcx_abort calls it (fcx_c_string turns the message into a string)
    FUNCTION fcx_set_abort_handler(handler) BIND(C, name='fcx_set_abort_handler')
      IMPORT :: c_int, c_funptr
      TYPE(c_funptr), VALUE :: handler
      INTEGER(c_int) :: fcx_set_abort_handler
    END FUNCTION
    FUNCTION fcx_abort(message) BIND(C, name='fcx_abort')
      IMPORT :: c_int, c_char
      CHARACTER(kind=c_char), DIMENSION(*), INTENT(IN) :: message
      INTEGER(c_int) :: fcx_abort
    END FUNCTION
    ! -- the rest of include/fcx.h: plan audit, streams, device memory, diagnostics --------
    FUNCTION fcx_plan_check(engine) BIND(C, name='fcx_plan_check')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int) :: fcx_plan_check
    END FUNCTION
    FUNCTION fcx_set_stream(engine, hip_stream) BIND(C, name='fcx_set_stream')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine, hip_stream
      INTEGER(c_int) :: fcx_set_stream
    END FUNCTION
    FUNCTION fcx_device_ptr(engine, surface_type, grid, var, dptr) BIND(C, name='fcx_device_ptr')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: surface_type, grid, var
      TYPE(c_ptr), INTENT(OUT) :: dptr
      INTEGER(c_int) :: fcx_device_ptr
    END FUNCTION
    FUNCTION fcx_device_layout(engine, tile, tile_stride) BIND(C, name='fcx_device_layout')
      IMPORT :: c_int, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int64_t), INTENT(OUT) :: tile, tile_stride
      INTEGER(c_int) :: fcx_device_layout
    END FUNCTION
    FUNCTION fcx_last_kernel_ms(engine, ms) BIND(C, name='fcx_last_kernel_ms')
      IMPORT :: c_int, c_float, c_ptr
      TYPE(c_ptr), VALUE :: engine
      REAL(c_float), INTENT(OUT) :: ms
      INTEGER(c_int) :: fcx_last_kernel_ms
    END FUNCTION
    FUNCTION fcx_span_runs(engine, phase, h2d_copies, d2h_copies) BIND(C, name='fcx_span_runs')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: phase
      INTEGER(c_int32_t), INTENT(OUT) :: h2d_copies, d2h_copies
      INTEGER(c_int) :: fcx_span_runs
    END FUNCTION
    FUNCTION fcx_algorithmic_bytes(engine, phase, bytes) BIND(C, name='fcx_algorithmic_bytes')
      IMPORT :: c_int, c_int64_t, c_ptr
      TYPE(c_ptr), VALUE :: engine
      INTEGER(c_int), VALUE :: phase
      INTEGER(c_int64_t), INTENT(OUT) :: bytes
      INTEGER(c_int) :: fcx_algorithmic_bytes
    END FUNCTION
    FUNCTION fcx_set_atmos_shared(engine, shared, n_boundaries, stride, left, right) &
        BIND(C, name='fcx_set_atmos_shared')
      IMPORT :: c_int, c_int32_t, c_ptr
      TYPE(c_ptr), VALUE :: engine, shared
      INTEGER(c_int32_t), VALUE :: n_boundaries, stride, left, right
      INTEGER(c_int) :: fcx_set_atmos_shared
    END FUNCTION
    FUNCTION fcx_comm_allreduce_sum(comm, buf, count, hip_stream) BIND(C, name='fcx_comm_allreduce_sum')
      IMPORT :: c_int, c_size_t, c_ptr
      TYPE(c_ptr), VALUE :: comm, buf, hip_stream
      INTEGER(c_size_t), VALUE :: count
      INTEGER(c_int) :: fcx_comm_allreduce_sum
    END FUNCTION
    FUNCTION fcx_atmos_allreduce(comm, engines, n_engines) BIND(C, name='fcx_atmos_allreduce')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: comm
      TYPE(c_ptr), DIMENSION(*), INTENT(IN) :: engines
      INTEGER(c_int), VALUE :: n_engines
      INTEGER(c_int) :: fcx_atmos_allreduce
    END FUNCTION
    FUNCTION fcx_device_malloc(device, bytes, ptr) BIND(C, name='fcx_device_malloc')
      IMPORT :: c_int, c_size_t, c_ptr
      INTEGER(c_int), VALUE :: device
      INTEGER(c_size_t), VALUE :: bytes
      TYPE(c_ptr), INTENT(OUT) :: ptr
      INTEGER(c_int) :: fcx_device_malloc
    END FUNCTION
    FUNCTION fcx_device_free(ptr) BIND(C, name='fcx_device_free')
      IMPORT :: c_int, c_ptr
      TYPE(c_ptr), VALUE :: ptr
      INTEGER(c_int) :: fcx_device_free
    END FUNCTION
    ! kind: 1 host->device, 2 device->host, 3 device->device (synchronous)
    FUNCTION fcx_memcpy(dst, src, bytes, kind) BIND(C, name='fcx_memcpy')
      IMPORT :: c_int, c_size_t, c_ptr
      TYPE(c_ptr), VALUE :: dst, src
      INTEGER(c_size_t), VALUE :: bytes
      INTEGER(c_int), VALUE :: kind
      INTEGER(c_int) :: fcx_memcpy
    END FUNCTION
  END INTERFACE

CONTAINS

  ! fcx_last_error() as a Fortran string
  FUNCTION fcx_error_message() RESULT(msg)
    CHARACTER(len=512) :: msg
    TYPE(c_ptr) :: p
    CHARACTER(kind=c_char), DIMENSION(:), POINTER :: chars
    INTEGER :: i
    msg = ''
    p = fcx_last_error()
    IF (.NOT. c_associated(p)) RETURN
    CALL c_f_pointer(p, chars, [512])
    DO i = 1, 512
      IF (chars(i) == c_null_char) EXIT
      msg(i:i) = chars(i)
    END DO
  END FUNCTION

  ! a NUL-terminated C string (an abort handler's argument) as a Fortran string
  FUNCTION fcx_c_string(chars) RESULT(msg)
    CHARACTER(kind=c_char), DIMENSION(*), INTENT(IN) :: chars
    CHARACTER(len=512) :: msg
    INTEGER :: i
    msg = ''
    DO i = 1, 512
      IF (chars(i) == c_null_char) EXIT
      msg(i:i) = chars(i)
    END DO
  END FUNCTION

  ! trim(method) of a CHARACTER(len=20) namelist entry -> enum fcx_method (-1 unknown)
  FUNCTION fcx_method_id(method) RESULT(id)
    CHARACTER(len=*), INTENT(IN) :: method
    INTEGER(c_int) :: id
    id = fcx_method_from_string(method, INT(LEN(method), c_size_t))
  END FUNCTION

END MODULE fcx_c_api
