! flux_calculator_calculate.F90 -- drop-in replacement of the reference module
! flux_calculator_calculate (/root/reference/src/flux_calculator_calculate.F90) that runs
! the flux path on an MI355X through libfcx (include/fcx.h).
!
! Same module name, same public subroutines, same arguments:
!   calc_spec_vapor_surface, calc_flux_mass_evap, calc_flux_heat_latent,
!   calc_flux_heat_sensible, calc_flux_momentum_east, calc_flux_momentum_north,
!   calc_flux_radiation_blackbody, distribute_shortwave_radiation_flux,
!   average_across_surface_types
! plus the engine life cycle the host calls once (INTEGRATION.md):
!   fcx_attach              after flux_calculator.F90:761 (all allocations/aliases final)
!   fcx_register_average    for each type-0 output (optional: fused averaging)
!   fcx_commit_engine       validate + device mirrors
!   fcx_run_phase           fused coupling-step phase (replaces :902 and :972-991)
!   fcx_start_phase /       the same phase in two halves: started (inputs taken, launch and
!   fcx_finish_phase        downloads queued), then completed (outputs in local_field), so
!                           the host can do other work -- e.g. an oasis_get -- in between
!   fcx_detach              at finalisation
! The per-call subroutines keep the reference's exact semantics (each uploads what it
! reads, computes on the GPU, downloads what it writes).  Errors are written to w_unit,
! handed to the host's abort routine when one is registered (fcx_register_abort: a routine
! that calls oasis_abort, as the reference does on a failed exchange, flux_calculator.F90:
! 883-887, so the other components do not wait forever in their next exchange) and stop
! the rank.
MODULE flux_calculator_calculate

    USE flux_calculator_basic
    USE fcx_c_api
    USE, INTRINSIC :: iso_c_binding

    IMPLICIT NONE
    PRIVATE

    PUBLIC calc_spec_vapor_surface
    PUBLIC calc_flux_mass_evap
    PUBLIC calc_flux_heat_latent
    PUBLIC calc_flux_heat_sensible
    PUBLIC calc_flux_momentum_east
    PUBLIC calc_flux_momentum_north
    PUBLIC calc_flux_radiation_blackbody
    PUBLIC distribute_shortwave_radiation_flux
    PUBLIC average_across_surface_types
    PUBLIC fcx_attach, fcx_register_average, fcx_commit_engine, fcx_run_phase, fcx_detach
    PUBLIC fcx_register_abort, fcx_start_phase, fcx_finish_phase, fcx_hand_over_field
    PUBLIC fcx_allocate_field, fcx_free_field

    TYPE(c_ptr), SAVE :: engine = c_null_ptr
    ! What fcx_attach bound.  The reference subroutines take the bottom model, the type count,
    ! the method table and grid_size on every call (calc:25-385); the engine takes them once.
    ! Each per-call subroutine checks its own arguments against these and stops with a named
    ! error when they differ or when no engine is attached.
    INTEGER, SAVE :: att_model = -1, att_types = -1, att_grid(3) = -1
    CHARACTER(len=20), SAVE :: att_methods(0:7, MAX_SURFACE_TYPES)

CONTAINS

    ! the host's abort routine: a BIND(C) subroutine with one argument
    ! CHARACTER(kind=c_char), DIMENSION(*) (the NUL-terminated message; fcx_c_string), passed
    ! as c_funloc(routine).  It is called before the rank stops; a routine that calls
    ! oasis_abort(comp_id, comp_name, fcx_c_string(msg)) ends the coupled job.
    SUBROUTINE fcx_register_abort(handler)
        TYPE(c_funptr), INTENT(IN) :: handler
        INTEGER(c_int) :: r
        r = fcx_set_abort_handler(handler)
    END SUBROUTINE fcx_register_abort

    ! Library memory for one local_field array (INTEGRATION.md section 3): the host calls this
    ! where the reference ALLOCATEs the array -- allocate_localvar (basic:288-309) for every
    ! input, do_prepare_calculation (prepare:36-42) for every output -- and frees it with
    ! fcx_free_field after fcx_detach.  fcx_host_malloc hands out consecutive blocks, so in
    ! the reference's order the inputs form one span and the outputs another, and each phase
    ! moves them with one copy per direction (FCX_OPT_LIB_SPANS).
    SUBROUTINE fcx_allocate_field(field, length)
        REAL(wp), POINTER, INTENT(INOUT) :: field(:)
        INTEGER,           INTENT(IN)    :: length
        TYPE(c_ptr) :: blk
        INTEGER(c_size_t) :: bytes
        bytes = INT(MAX(length, 1), c_size_t) * INT(STORAGE_SIZE(1.0_wp) / 8, c_size_t)
        CALL check(fcx_host_malloc(bytes, blk), 'fcx_allocate_field')
        CALL C_F_POINTER(blk, field, [length])
    END SUBROUTINE fcx_allocate_field

    SUBROUTINE fcx_free_field(field)
        REAL(wp), POINTER, INTENT(INOUT) :: field(:)
        IF (.NOT. ASSOCIATED(field)) RETURN
        IF (SIZE(field) > 0) CALL check(fcx_host_free(C_LOC(field(1))), 'fcx_free_field')
        NULLIFY (field)
    END SUBROUTINE fcx_free_field

    ! the end of the rank on an error: message to w_unit, the host's abort routine, stop
    SUBROUTINE stop_run(msg)
        CHARACTER(len=*), INTENT(IN) :: msg
        INTEGER(c_int) :: r
        WRITE (w_unit, '(A)') msg
        CALL FLUSH(w_unit)
        r = fcx_abort(msg // c_null_char)  ! FCX_E_STATE when no routine is registered
        ERROR STOP 1
    END SUBROUTINE stop_run

    SUBROUTINE check(status, where)
        INTEGER(c_int),   INTENT(IN) :: status
        CHARACTER(len=*), INTENT(IN) :: where
        IF (status /= FCX_OK) CALL stop_run('flux engine error in ' // where // ': ' // TRIM(fcx_error_message()))
    END SUBROUTINE check

    SUBROUTINE contract_error(where, msg)
        CHARACTER(len=*), INTENT(IN) :: where, msg
        CALL stop_run('flux engine contract violation in ' // where // ': ' // msg)
    END SUBROUTINE contract_error

    ! the per-call subroutine `where` against the attached engine: an engine exists, and
    ! num_surface_types, grid_size(1:3), my_bottom_model and its method table column are the
    ! ones fcx_attach bound (flux: FCX_* table id; absent for calls that take no table)
    SUBROUTINE require(where, num_surface_types, grid_size, my_bottom_model, flux, methods)
        CHARACTER(len=*),                            INTENT(IN) :: where
        INTEGER,                                     INTENT(IN) :: num_surface_types
        INTEGER,           DIMENSION(:),             INTENT(IN) :: grid_size
        INTEGER,                           OPTIONAL, INTENT(IN) :: my_bottom_model
        INTEGER(c_int),                    OPTIONAL, INTENT(IN) :: flux
        CHARACTER(len=20), DIMENSION(:,:), OPTIONAL, INTENT(IN) :: methods
        CHARACTER(len=256) :: msg
        INTEGER :: i
        IF (.NOT. c_associated(engine)) CALL contract_error(where, &
            'no flux engine attached (call fcx_attach once all fields are allocated, after flux_calculator.F90:761)')
        IF (num_surface_types /= att_types) THEN
            WRITE (msg, '(A,I0,A,I0)') 'num_surface_types ', num_surface_types, ' but the engine was attached with ', &
                att_types
            CALL contract_error(where, TRIM(msg))
        ENDIF
        IF (SIZE(grid_size) < 3) CALL contract_error(where, 'grid_size has fewer than 3 grids')
        IF (ANY(grid_size(1:3) /= att_grid)) THEN
            WRITE (msg, '(A,3(1X,I0),A,3(1X,I0))') 'grid_size', grid_size(1:3), ' but the engine was attached with', &
                att_grid
            CALL contract_error(where, TRIM(msg))
        ENDIF
        IF (PRESENT(my_bottom_model)) THEN
            IF (my_bottom_model /= att_model) THEN
                WRITE (msg, '(A,I0,A,I0)') 'my_bottom_model ', my_bottom_model, ' but the engine was attached with ', &
                    att_model
                CALL contract_error(where, TRIM(msg))
            ENDIF
        ENDIF
        IF (PRESENT(methods) .AND. PRESENT(flux) .AND. PRESENT(my_bottom_model)) THEN
            DO i = 1, num_surface_types
                IF (TRIM(methods(my_bottom_model, i)) /= TRIM(att_methods(flux, i))) THEN
                    WRITE (msg, '(A,I0,5A)') 'method table differs from the attached one: surface type ', i, &
                        ' is "', TRIM(methods(my_bottom_model, i)), '", attached "', TRIM(att_methods(flux, i)), '"'
                    CALL contract_error(where, TRIM(msg))
                ENDIF
            ENDDO
        ENDIF
    END SUBROUTINE require

    SUBROUTINE set_table(flux, methods, my_bottom_model, num_surface_types)
        INTEGER(c_int),                          INTENT(IN) :: flux
        CHARACTER(len=20), DIMENSION(:,:),       INTENT(IN) :: methods
        INTEGER,                                 INTENT(IN) :: my_bottom_model, num_surface_types
        INTEGER :: i
        INTEGER(c_int) :: m
        DO i = 1, num_surface_types
            m = fcx_method_id(methods(my_bottom_model, i))
            IF (m < 0) CALL stop_run('Method ' // TRIM(methods(my_bottom_model, i)) // ' is not known.')
            CALL check(fcx_set_method(engine, flux, INT(i, c_int), m), 'fcx_set_method')
            att_methods(flux, i) = methods(my_bottom_model, i)
        ENDDO
    END SUBROUTINE set_table

    ! Bind every ASSOCIATED local_field slot (aliases = identical addresses), the method
    ! tables, the bias corrections and the rank-local regridding matrices.
    SUBROUTINE fcx_attach(my_bottom_model, num_surface_types, grid_size, local_field,          &
                          which_spec_vapor_surface_t, which_spec_vapor_surface_u,            &
                          which_spec_vapor_surface_v, which_flux_mass_evap,                  &
                          which_flux_heat_latent, which_flux_heat_sensible,                  &
                          which_flux_momentum, which_flux_radiation_blackbody,               &
                          lcorrection, correction_init_date, corrections_mass_evap,          &
                          regrid_u_to_t_matrix, regrid_v_to_t_matrix,                        &
                          regrid_t_to_u_matrix, regrid_t_to_v_matrix, device)
        INTEGER,                                  INTENT(IN) :: my_bottom_model, num_surface_types
        INTEGER,                 DIMENSION(:),    INTENT(IN) :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(IN), TARGET :: local_field
        CHARACTER(len=20),       DIMENSION(:,:),  INTENT(IN) :: which_spec_vapor_surface_t, &
            which_spec_vapor_surface_u, which_spec_vapor_surface_v, which_flux_mass_evap,    &
            which_flux_heat_latent, which_flux_heat_sensible, which_flux_momentum,           &
            which_flux_radiation_blackbody
        LOGICAL,                                  INTENT(IN) :: lcorrection
        INTEGER,                                  INTENT(IN) :: correction_init_date
        REAL(kind=wp), DIMENSION(:,:), TARGET,    INTENT(IN), OPTIONAL :: corrections_mass_evap ! (12, grid_size(1))
        TYPE(sparse_regridding_matrix),           INTENT(IN), OPTIONAL, TARGET :: regrid_u_to_t_matrix, &
            regrid_v_to_t_matrix, regrid_t_to_u_matrix, regrid_t_to_v_matrix
        INTEGER,                                  INTENT(IN), OPTIONAL :: device
        INTEGER(c_int32_t) :: gs(3)
        INTEGER(c_int) :: dev, flags, mask
        INTEGER :: s, g, v
        REAL(c_double), ALLOCATABLE, TARGET :: corr_d(:,:)

        IF (c_associated(engine)) CALL fcx_detach()
        gs = INT(grid_size(1:3), c_int32_t)
        att_model = my_bottom_model
        att_types = num_surface_types
        att_grid = grid_size(1:3)
        att_methods = ''
        dev = 0
        IF (PRESENT(device)) dev = INT(device, c_int)
        CALL check(fcx_create(dev, INT(num_surface_types, c_int), gs, engine), 'fcx_create')
        ! the NO_USE_DOUBLE_PRECISION build (basic:21-25) keeps REAL(4) fields: fp32 engine
        IF (wp == c_float) CALL check(fcx_set_precision(engine, FCX_PRECISION_F32), 'fcx_set_precision')

        CALL set_table(FCX_SPEC_VAPOR_SURFACE_T, which_spec_vapor_surface_t, my_bottom_model, num_surface_types)
        CALL set_table(FCX_SPEC_VAPOR_SURFACE_U, which_spec_vapor_surface_u, my_bottom_model, num_surface_types)
        CALL set_table(FCX_SPEC_VAPOR_SURFACE_V, which_spec_vapor_surface_v, my_bottom_model, num_surface_types)
        CALL set_table(FCX_FLUX_MASS_EVAP, which_flux_mass_evap, my_bottom_model, num_surface_types)
        CALL set_table(FCX_FLUX_HEAT_LATENT, which_flux_heat_latent, my_bottom_model, num_surface_types)
        CALL set_table(FCX_FLUX_HEAT_SENSIBLE, which_flux_heat_sensible, my_bottom_model, num_surface_types)
        CALL set_table(FCX_FLUX_MOMENTUM, which_flux_momentum, my_bottom_model, num_surface_types)
        CALL set_table(FCX_FLUX_RADIATION_BLACKBODY, which_flux_radiation_blackbody, my_bottom_model, &
                       num_surface_types)

        ! local_field(0:MAX_SURFACE_TYPES, 3)%var(MAX_VARNAMES) (flux_calculator.F90:159)
        DO s = 0, MAX_SURFACE_TYPES
            DO g = 1, 3
                DO v = 1, MAX_VARNAMES
                    IF (.NOT. ASSOCIATED(local_field(s,g)%var(v)%field)) CYCLE
                    IF (SIZE(local_field(s,g)%var(v)%field) == 0) CYCLE
                    flags = FCX_MEM_HOST
                    IF (local_field(s,g)%var(v)%allocated) flags = IOR(flags, FCX_ALLOCATED)
                    CALL check(fcx_bind_field(engine, INT(s, c_int), INT(g, c_int), INT(v, c_int),  &
                                              c_loc(local_field(s,g)%var(v)%field(1)),          &
                                              INT(SIZE(local_field(s,g)%var(v)%field), c_int64_t), &
                                              flags), 'fcx_bind_field')
                    mask = 0
                    IF (local_field(s,g)%var(v)%put_to_t_grid) mask = IOR(mask, 1)
                    IF (local_field(s,g)%var(v)%put_to_u_grid) mask = IOR(mask, 2)
                    IF (local_field(s,g)%var(v)%put_to_v_grid) mask = IOR(mask, 4)
                    IF (mask /= 0) CALL check(fcx_set_put_to(engine, INT(s, c_int), INT(g, c_int), &
                                                             INT(v, c_int), mask), 'fcx_set_put_to')
                ENDDO
            ENDDO
        ENDDO

        ! bias_corrections: corrections(E_MASS_EVAP_CORRECTION, :, :) is (12, grid_size(1))
        IF (lcorrection .AND. PRESENT(corrections_mass_evap)) THEN
            ! the C ABI takes the corrections as double (copied at the call)
            corr_d = REAL(corrections_mass_evap, c_double)
            CALL check(fcx_set_corrections(engine, 1_c_int, INT(correction_init_date, c_int32_t),  &
                                           c_loc(corr_d(1,1)),                                   &
                                           INT(grid_size(1), c_int64_t), FCX_CORR_CELL_MAJOR),    &
                       'fcx_set_corrections')
            DEALLOCATE(corr_d)
        ENDIF

        IF (PRESENT(regrid_u_to_t_matrix)) CALL set_matrix(FCX_U_TO_T, regrid_u_to_t_matrix)
        IF (PRESENT(regrid_v_to_t_matrix)) CALL set_matrix(FCX_V_TO_T, regrid_v_to_t_matrix)
        IF (PRESENT(regrid_t_to_u_matrix)) CALL set_matrix(FCX_T_TO_U, regrid_t_to_u_matrix)
        IF (PRESENT(regrid_t_to_v_matrix)) CALL set_matrix(FCX_T_TO_V, regrid_t_to_v_matrix)
    END SUBROUTINE fcx_attach

    SUBROUTINE set_matrix(which, m)
        INTEGER(c_int),                         INTENT(IN) :: which
        TYPE(sparse_regridding_matrix), TARGET, INTENT(IN) :: m
        ! the C ABI takes double weights (copied at the call); REAL(wp) may be REAL(4)
        REAL(c_double), ALLOCATABLE, TARGET :: w8(:)
        IF (m%num_elements <= 0) RETURN
        ALLOCATE(w8(m%num_elements))
        w8 = REAL(m%weight%field(1:m%num_elements), c_double)
        CALL check(fcx_set_regrid_matrix(engine, which, INT(m%num_elements, c_int64_t),          &
                                         c_loc(m%src_index%field(1)), c_loc(m%dst_index%field(1)), &
                                         c_loc(w8(1))), 'fcx_set_regrid_matrix')
        DEALLOCATE(w8)
    END SUBROUTINE set_matrix

    ! output_field(j) with surface_type 0 (flux_calculator.F90:909-918, 999-1008)
    SUBROUTINE fcx_register_average(early, which_grid, my_idx)
        LOGICAL, INTENT(IN) :: early
        INTEGER, INTENT(IN) :: which_grid, my_idx
        INTEGER(c_int) :: phase
        phase = FCX_PHASE_NORMAL
        IF (early) phase = FCX_PHASE_EARLY
        CALL check(fcx_add_average(engine, phase, INT(which_grid, c_int), INT(my_idx, c_int)), &
                   'fcx_add_average')
    END SUBROUTINE fcx_register_average

    ! every plan the engine can launch audited on the host first (fcx_plan_check: a method
    ! that would read an input the set-up left unbound stops here with a named error, before
    ! any device memory is taken), then validation and the device mirrors
    SUBROUTINE fcx_commit_engine()
        CALL check(fcx_plan_check(engine), 'fcx_plan_check')
        CALL check(fcx_commit(engine), 'fcx_commit')
    END SUBROUTINE fcx_commit_engine

    ! One fused phase: upload the phase's inputs, all its fluxes + regrids + type-0
    ! averages in one pass, download its outputs.  phase: FCX_PHASE_EARLY (replaces
    ! flux_calculator.F90:902-918) or FCX_PHASE_NORMAL (replaces :972-1008).
    SUBROUTINE fcx_run_phase(phase)
        INTEGER(c_int), INTENT(IN) :: phase
        CALL check(fcx_step(engine, phase, INT(current_step_time, c_int32_t)), 'fcx_step')
    END SUBROUTINE fcx_run_phase

    ! fcx_run_phase in two halves (fcx_step_async + fcx_synchronize): after fcx_start_phase
    ! the phase's input fields may be overwritten (their values are in the engine); its
    ! output fields hold the results after fcx_finish_phase
    SUBROUTINE fcx_start_phase(phase)
        INTEGER(c_int), INTENT(IN) :: phase
        CALL check(fcx_step_async(engine, phase, INT(current_step_time, c_int32_t)), 'fcx_step_async')
    END SUBROUTINE fcx_start_phase

    ! one input field right after its oasis_get (flux_calculator.F90:876-880, 946-950): the
    ! engine's upload thread stages it while the host receives the next field; the phase that
    ! follows moves only the inputs not handed over.  The array may be overwritten once the
    ! next engine call returns.
    SUBROUTINE fcx_hand_over_field(surface_type, which_grid, my_idx)
        INTEGER, INTENT(IN) :: surface_type, which_grid, my_idx
        CALL check(fcx_upload_field(engine, INT(surface_type, c_int), INT(which_grid, c_int), INT(my_idx, c_int)), &
                   'fcx_upload_field')
    END SUBROUTINE fcx_hand_over_field

    SUBROUTINE fcx_finish_phase()
        CALL check(fcx_synchronize(engine), 'fcx_synchronize')
    END SUBROUTINE fcx_finish_phase

    SUBROUTINE fcx_detach()
        INTEGER(c_int) :: r
        IF (.NOT. c_associated(engine)) RETURN
        r = fcx_destroy(engine)
        engine = c_null_ptr
        att_model = -1
        att_types = -1
        att_grid = -1
    END SUBROUTINE fcx_detach

    !!!!!!!!!! the reference subroutines (flux_calculator_calculate.F90:25-385) !!!!!!!!!!

    SUBROUTINE calc_spec_vapor_surface(my_bottom_model, num_surface_types, which_grid, methods, grid_size, local_field)
        INTEGER,                                  INTENT(IN)    :: my_bottom_model
        INTEGER,                                  INTENT(IN)    :: num_surface_types
        INTEGER,                                  INTENT(IN)    :: which_grid
        CHARACTER(len=20),       DIMENSION(:,:),  INTENT(IN)    :: methods
        INTEGER,                 DIMENSION(:),    INTENT(IN)    :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(INOUT) :: local_field
        IF (which_grid < 1 .OR. which_grid > 3) CALL contract_error('calc_spec_vapor_surface', 'which_grid outside 1..3')
        CALL require('calc_spec_vapor_surface', num_surface_types, grid_size, my_bottom_model, &
                     FCX_SPEC_VAPOR_SURFACE_T + INT(which_grid - 1, c_int), methods)
        CALL check(fcx_calc_spec_vapor_surface(engine, INT(which_grid, c_int)), 'calc_spec_vapor_surface')
    END SUBROUTINE calc_spec_vapor_surface

    SUBROUTINE calc_flux_mass_evap(my_bottom_model, num_surface_types, methods, grid_size, local_field)
        INTEGER,                                  INTENT(IN)    :: my_bottom_model
        INTEGER,                                  INTENT(IN)    :: num_surface_types
        CHARACTER(len=20),       DIMENSION(:,:),  INTENT(IN)    :: methods
        INTEGER,                 DIMENSION(:),    INTENT(IN)    :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(INOUT) :: local_field
        ! the month of the bias correction comes from current_step_time (basic:125)
        CALL require('calc_flux_mass_evap', num_surface_types, grid_size, my_bottom_model, FCX_FLUX_MASS_EVAP, methods)
        CALL check(fcx_calc_flux_mass_evap(engine, INT(current_step_time, c_int32_t)), 'calc_flux_mass_evap')
    END SUBROUTINE calc_flux_mass_evap

    SUBROUTINE calc_flux_heat_latent(my_bottom_model, num_surface_types, methods, grid_size, local_field)
        INTEGER,                                  INTENT(IN)    :: my_bottom_model
        INTEGER,                                  INTENT(IN)    :: num_surface_types
        CHARACTER(len=20),       DIMENSION(:,:),  INTENT(IN)    :: methods
        INTEGER,                 DIMENSION(:),    INTENT(IN)    :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(INOUT) :: local_field
        CALL require('calc_flux_heat_latent', num_surface_types, grid_size, my_bottom_model, FCX_FLUX_HEAT_LATENT, &
                     methods)
        CALL check(fcx_calc_flux_heat_latent(engine), 'calc_flux_heat_latent')
    END SUBROUTINE calc_flux_heat_latent

    SUBROUTINE calc_flux_heat_sensible(my_bottom_model, num_surface_types, methods, grid_size, local_field)
        INTEGER,                                  INTENT(IN)    :: my_bottom_model
        INTEGER,                                  INTENT(IN)    :: num_surface_types
        CHARACTER(len=20),       DIMENSION(:,:),  INTENT(IN)    :: methods
        INTEGER,                 DIMENSION(:),    INTENT(IN)    :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(INOUT) :: local_field
        CALL require('calc_flux_heat_sensible', num_surface_types, grid_size, my_bottom_model, &
                     FCX_FLUX_HEAT_SENSIBLE, methods)
        CALL check(fcx_calc_flux_heat_sensible(engine), 'calc_flux_heat_sensible')
    END SUBROUTINE calc_flux_heat_sensible

    SUBROUTINE calc_flux_momentum_east(my_bottom_model, num_surface_types, which_grid, methods, grid_size, local_field)
        INTEGER,                                  INTENT(IN)    :: my_bottom_model
        INTEGER,                                  INTENT(IN)    :: num_surface_types
        INTEGER,                                  INTENT(IN)    :: which_grid
        CHARACTER(len=20),       DIMENSION(:,:),  INTENT(IN)    :: methods
        INTEGER,                 DIMENSION(:),    INTENT(IN)    :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(INOUT) :: local_field
        CALL require('calc_flux_momentum_east', num_surface_types, grid_size, my_bottom_model, FCX_FLUX_MOMENTUM, &
                     methods)
        CALL check(fcx_calc_flux_momentum_east(engine, INT(which_grid, c_int)), 'calc_flux_momentum_east')
    END SUBROUTINE calc_flux_momentum_east

    SUBROUTINE calc_flux_momentum_north(my_bottom_model, num_surface_types, which_grid, methods, grid_size, local_field)
        INTEGER,                                  INTENT(IN)    :: my_bottom_model
        INTEGER,                                  INTENT(IN)    :: num_surface_types
        INTEGER,                                  INTENT(IN)    :: which_grid
        CHARACTER(len=20),       DIMENSION(:,:),  INTENT(IN)    :: methods
        INTEGER,                 DIMENSION(:),    INTENT(IN)    :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(INOUT) :: local_field
        CALL require('calc_flux_momentum_north', num_surface_types, grid_size, my_bottom_model, FCX_FLUX_MOMENTUM, &
                     methods)
        CALL check(fcx_calc_flux_momentum_north(engine, INT(which_grid, c_int)), 'calc_flux_momentum_north')
    END SUBROUTINE calc_flux_momentum_north

    SUBROUTINE calc_flux_radiation_blackbody(my_bottom_model, num_surface_types, methods, grid_size, local_field)
        INTEGER,                                  INTENT(IN)    :: my_bottom_model
        INTEGER,                                  INTENT(IN)    :: num_surface_types
        CHARACTER(len=20),       DIMENSION(:,:),  INTENT(IN)    :: methods
        INTEGER,                 DIMENSION(:),    INTENT(IN)    :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(INOUT) :: local_field
        CALL require('calc_flux_radiation_blackbody', num_surface_types, grid_size, my_bottom_model, &
                     FCX_FLUX_RADIATION_BLACKBODY, methods)
        CALL check(fcx_calc_flux_radiation_blackbody(engine), 'calc_flux_radiation_blackbody')
    END SUBROUTINE calc_flux_radiation_blackbody

    SUBROUTINE distribute_shortwave_radiation_flux(my_bottom_model, num_surface_types, grid_size, local_field)
        INTEGER,                                  INTENT(IN)    :: my_bottom_model
        INTEGER,                                  INTENT(IN)    :: num_surface_types
        INTEGER,                 DIMENSION(:),    INTENT(IN)    :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(INOUT) :: local_field
        CALL require('distribute_shortwave_radiation_flux', num_surface_types, grid_size, my_bottom_model)
        CALL check(fcx_distribute_shortwave_radiation_flux(engine), 'distribute_shortwave_radiation_flux')
    END SUBROUTINE distribute_shortwave_radiation_flux

    SUBROUTINE average_across_surface_types(which_grid, my_idx, num_surface_types, grid_size, local_field)
        INTEGER,                                  INTENT(IN)    :: which_grid
        INTEGER,                                  INTENT(IN)    :: my_idx
        INTEGER,                                  INTENT(IN)    :: num_surface_types
        INTEGER,                 DIMENSION(:),    INTENT(IN)    :: grid_size
        TYPE(local_fields_type), DIMENSION(0:,:), INTENT(INOUT) :: local_field
        CALL require('average_across_surface_types', num_surface_types, grid_size)
        CALL check(fcx_average_across_surface_types(engine, INT(which_grid, c_int), INT(my_idx, c_int)), &
                   'average_across_surface_types')
    END SUBROUTINE average_across_surface_types

END MODULE flux_calculator_calculate
