! dropin_host.F90 -- a Fortran host of the drop-in module (test harness, not the product).
!
! It plays the reference main program (flux_calculator.F90) around the flux path: the
! reference's own data-model module flux_calculator_basic (compiled unmodified from the
! reference sources into oracle/_ref/mod by oracle/Makefile) holds local_field, and the
! drop-in module flux_calculator_calculate (components.flux_calculator_amd/fortran) is
! called with the reference's argument lists, in the order of flux_calculator.F90:902-1008.
! No regridding matrices are set, so the reference's do_regridding calls between the
! calc_* calls would be no-ops and are left out.
!
!   dropin_host <dir> percall|fused|async|handover|libmem|libmem_async|noattach|badtable|badgrid|badtypes[+abort]
!
! libmem / libmem_async: every buffer allocated with fcx_allocate_field (library memory,
! INTEGRATION.md section 3) in manifest order -- inputs, then outputs, as the reference
! allocates them -- and the fused phases (started and finished) run on the span transport.
!
! handover: before each fused phase every bound input field is handed over one by one
! (fcx_hand_over_field, as after each oasis_get), then the phase runs.
!
! +abort: the host registers its abort routine (fcx_register_abort) first, as a coupled
! host registers one that calls oasis_abort; this one prints the message and stops with 3.
!
! <dir>/manifest.txt (written by tests/test_fortran.py), one record per line:
!   N nbufs T nt nu nv          buffer count, surface types, grid sizes
!   A k n file                  buffer k: n REAL(8) values (stream file)
!   S s g v k alloc             local_field(s,g)%var(v)%field => buffer k (aliases share k)
!   M table s method            which_* table (1..8, fcx_attach order) of surface type s
!   C init_date file            bias corrections (12, nt), REAL(8), lcorrections = .TRUE.
!   V phase g v                 type-0 output (average_across_surface_types), phase 1 early
!   R seconds                   current_step_time
!   O s g v file                output written back after the step
PROGRAM dropin_host
    USE flux_calculator_basic
    USE flux_calculator_calculate
    USE fcx_c_api, ONLY: FCX_PHASE_EARLY, FCX_PHASE_NORMAL
    USE, INTRINSIC :: iso_c_binding, ONLY: c_funloc, c_char
    IMPLICIT NONE
    INTERFACE
        SUBROUTINE host_abort(msg) BIND(C)
            IMPORT :: c_char
            CHARACTER(kind=c_char), DIMENSION(*), INTENT(IN) :: msg
        END SUBROUTINE host_abort
    END INTERFACE

    TYPE buf_t
        REAL(wp), POINTER :: p(:) => NULL()
    END TYPE buf_t
    TYPE(local_fields_type), TARGET :: local_field(0:MAX_SURFACE_TYPES, 3)
    TYPE(buf_t), ALLOCATABLE :: bufs(:)
    CHARACTER(len=20) :: tables(MAX_BOTTOM_MODELS, MAX_SURFACE_TYPES, 8)
    INTEGER :: grid_size(3), nsurf, nbufs, k, n, s, g, v, alloc, tbl, ph, init_date, ios, u, i
    INTEGER :: nav, nout
    INTEGER :: av(3, 100), outs(3, 200)
    CHARACTER(len=512) :: outpath(200)
    REAL(wp), ALLOCATABLE, TARGET :: corr(:,:)
    REAL(8), ALLOCATABLE :: tmp(:)
    LOGICAL :: lcorr
    CHARACTER(len=1024) :: dir, mode, line, path
    CHARACTER(len=4) :: tag
    CHARACTER(len=20) :: meth

    CALL get_command_argument(1, dir)
    CALL get_command_argument(2, mode)
    IF (INDEX(mode, '+abort') > 0) THEN
        CALL fcx_register_abort(c_funloc(host_abort))
        mode = mode(1:INDEX(mode, '+abort') - 1)
    ENDIF
    w_unit = 6
    CALL init_varname_idx
    DO s = 0, MAX_SURFACE_TYPES
        DO g = 1, 3
            CALL nullify_localvars(local_field(s, g))
        ENDDO
    ENDDO
    tables = 'none'
    lcorr = .FALSE.
    init_date = 0
    nav = 0
    nout = 0

    OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/manifest.txt', STATUS='old', ACTION='read')
    DO
        READ (u, '(A)', IOSTAT=ios) line
        IF (ios /= 0) EXIT
        READ (line, *) tag
        SELECT CASE (TRIM(tag))
        CASE ('N')
            READ (line, *) tag, nbufs, nsurf, grid_size(1), grid_size(2), grid_size(3)
            ALLOCATE (bufs(nbufs))
        CASE ('A')
            READ (line, *) tag, k, n, path
            IF (INDEX(mode, 'libmem') == 1) THEN
                CALL fcx_allocate_field(bufs(k)%p, n)
                ALLOCATE (tmp(n))
            ELSE
                ALLOCATE (bufs(k)%p(n), tmp(n))
            ENDIF
            CALL read_raw(TRIM(dir)//'/'//TRIM(path), tmp)
            bufs(k)%p = REAL(tmp, wp)
            DEALLOCATE (tmp)
        CASE ('S')
            READ (line, *) tag, s, g, v, k, alloc
            local_field(s, g)%var(v)%field => bufs(k)%p
            local_field(s, g)%var(v)%allocated = alloc == 1
        CASE ('M')
            READ (line, *) tag, tbl, s, meth
            tables(1, s, tbl) = meth
        CASE ('C')
            READ (line, *) tag, init_date, path
            ALLOCATE (corr(12, grid_size(1)), tmp(12 * grid_size(1)))
            CALL read_raw(TRIM(dir)//'/'//TRIM(path), tmp)
            corr = RESHAPE(REAL(tmp, wp), [12, grid_size(1)])
            DEALLOCATE (tmp)
            lcorr = .TRUE.
        CASE ('V')
            nav = nav + 1
            READ (line, *) tag, av(1, nav), av(2, nav), av(3, nav)
        CASE ('R')
            READ (line, *) tag, current_step_time
        CASE ('O')
            nout = nout + 1
            READ (line, *) tag, outs(1, nout), outs(2, nout), outs(3, nout), outpath(nout)
        END SELECT
    ENDDO
    CLOSE (u)

    ! contract checks of the per-call subroutines (no GPU work reaches the engine):
    ! the reference host loop without fcx_attach, and calls whose arguments differ from the
    ! attached ones -- each must stop with a named error
    IF (TRIM(mode) == 'noattach') CALL calc_flux_mass_evap(1, nsurf, tables(:,:,4), grid_size, local_field)

    ! after flux_calculator.F90:761: every allocation and alias is final
    IF (lcorr) THEN
        CALL fcx_attach(1, nsurf, grid_size, local_field, tables(:,:,1), tables(:,:,2), tables(:,:,3),   &
                        tables(:,:,4), tables(:,:,5), tables(:,:,6), tables(:,:,7), tables(:,:,8),    &
                        lcorr, init_date, corr)
    ELSE
        CALL fcx_attach(1, nsurf, grid_size, local_field, tables(:,:,1), tables(:,:,2), tables(:,:,3),   &
                        tables(:,:,4), tables(:,:,5), tables(:,:,6), tables(:,:,7), tables(:,:,8),    &
                        lcorr, init_date)
    ENDIF

    IF (TRIM(mode) == 'badtable') THEN
        IF (TRIM(tables(1, 1, 4)) == 'CCLM') THEN
            tables(1, 1, 4) = 'MOM5'
        ELSE
            tables(1, 1, 4) = 'CCLM'
        ENDIF
        CALL calc_flux_mass_evap(1, nsurf, tables(:,:,4), grid_size, local_field)
    ELSE IF (TRIM(mode) == 'badgrid') THEN
        CALL calc_flux_heat_latent(1, nsurf, tables(:,:,5), grid_size + [1, 0, 0], local_field)
    ELSE IF (TRIM(mode) == 'badtypes') THEN
        CALL average_across_surface_types(1, 22, nsurf + 1, grid_size, local_field)
    ENDIF

    IF (TRIM(mode) == 'fused' .OR. TRIM(mode) == 'async' .OR. TRIM(mode) == 'handover' .OR. &
        INDEX(mode, 'libmem') == 1) THEN
        ! INTEGRATION.md: two phases replace :902-918 and :972-1008
        DO i = 1, nav
            CALL fcx_register_average(av(1, i) == 1, av(2, i), av(3, i))
        ENDDO
        CALL fcx_commit_engine()
        IF (TRIM(mode) == 'handover') THEN
            CALL hand_over_inputs()
            CALL fcx_run_phase(FCX_PHASE_EARLY)
            CALL hand_over_inputs()
            CALL fcx_run_phase(FCX_PHASE_NORMAL)
        ELSE IF (TRIM(mode) == 'async' .OR. TRIM(mode) == 'libmem_async') THEN
            ! each phase started, then finished; the early phase's outputs are complete
            ! before the normal phase starts (its oasis_put precedes the normal oasis_get)
            CALL fcx_start_phase(FCX_PHASE_EARLY)
            CALL fcx_finish_phase()
            CALL fcx_start_phase(FCX_PHASE_NORMAL)
            CALL fcx_finish_phase()
        ELSE
            CALL fcx_run_phase(FCX_PHASE_EARLY)
            CALL fcx_run_phase(FCX_PHASE_NORMAL)
        ENDIF
    ELSE
        CALL fcx_commit_engine()
        ! flux_calculator.F90:902 and the early type-0 outputs (:909-918, P7 trigger)
        CALL calc_flux_radiation_blackbody(1, nsurf, tables(:,:,8), grid_size, local_field)
        CALL averages(1)
        ! :972-991
        CALL calc_spec_vapor_surface(1, nsurf, 1, tables(:,:,1), grid_size, local_field)
        CALL calc_spec_vapor_surface(1, nsurf, 2, tables(:,:,2), grid_size, local_field)
        CALL calc_spec_vapor_surface(1, nsurf, 3, tables(:,:,3), grid_size, local_field)
        CALL calc_flux_mass_evap(1, nsurf, tables(:,:,4), grid_size, local_field)
        CALL calc_flux_heat_latent(1, nsurf, tables(:,:,5), grid_size, local_field)
        CALL calc_flux_heat_sensible(1, nsurf, tables(:,:,6), grid_size, local_field)
        CALL calc_flux_momentum_east(1, nsurf, 2, tables(:,:,7), grid_size, local_field)
        CALL calc_flux_momentum_north(1, nsurf, 3, tables(:,:,7), grid_size, local_field)
        CALL distribute_shortwave_radiation_flux(1, nsurf, grid_size, local_field)
        ! :999-1008
        CALL averages(2)
    ENDIF
    CALL fcx_detach()

    DO i = 1, nout
        s = outs(1, i)
        g = outs(2, i)
        v = outs(3, i)
        CALL write_raw(TRIM(dir)//'/'//TRIM(outpath(i)), REAL(local_field(s, g)%var(v)%field, 8))
    ENDDO
    IF (INDEX(mode, 'libmem') == 1) THEN
        DO k = 1, nbufs
            CALL fcx_free_field(bufs(k)%p)
        ENDDO
    ENDIF
    WRITE (*, '(A)') 'DROPIN_HOST OK'

CONTAINS

    ! every bound field that no flux writes, handed over one by one as the host would after
    ! each oasis_get
    SUBROUTINE hand_over_inputs()
        INTEGER :: ss, gg, vv
        DO ss = 0, MAX_SURFACE_TYPES
            DO gg = 1, 3
                DO vv = 1, MAX_VARNAMES
                    IF (.NOT. ASSOCIATED(local_field(ss, gg)%var(vv)%field)) CYCLE
                    IF (ANY(vv == [idx_QSUR, idx_MEVA, idx_HLAT, idx_HSEN, idx_RBBR, idx_UMOM, idx_VMOM, &
                                   idx_RSDR])) CYCLE
                    CALL fcx_hand_over_field(ss, gg, vv)
                ENDDO
            ENDDO
        ENDDO
    END SUBROUTINE hand_over_inputs

    ! the P7 trigger of the main program: the type-0 slot is associated and surface type 2 exists
    SUBROUTINE averages(phase)
        INTEGER, INTENT(IN) :: phase
        INTEGER :: j
        DO j = 1, nav
            IF (av(1, j) /= phase) CYCLE
            IF (.NOT. ASSOCIATED(local_field(0, av(2, j))%var(av(3, j))%field)) CYCLE
            IF (nsurf < 2) CYCLE
            CALL average_across_surface_types(av(2, j), av(3, j), nsurf, grid_size, local_field)
        ENDDO
    END SUBROUTINE averages

    SUBROUTINE read_raw(fname, x)
        CHARACTER(len=*), INTENT(IN) :: fname
        REAL(8), INTENT(OUT) :: x(:)
        INTEGER :: uu
        OPEN (NEWUNIT=uu, FILE=fname, ACCESS='stream', FORM='unformatted', STATUS='old', ACTION='read')
        READ (uu) x
        CLOSE (uu)
    END SUBROUTINE read_raw

    SUBROUTINE write_raw(fname, x)
        CHARACTER(len=*), INTENT(IN) :: fname
        REAL(8), INTENT(IN) :: x(:)
        INTEGER :: uu
        OPEN (NEWUNIT=uu, FILE=fname, ACCESS='stream', FORM='unformatted', STATUS='replace', ACTION='write')
        WRITE (uu) x
        CLOSE (uu)
    END SUBROUTINE write_raw

END PROGRAM dropin_host

! The host program's MPI finalisation: flux_calculator_basic calls mpi_finalize(1) on a
! configuration error (basic:305 etc.); the real host links MPI, this single-rank test host
! has none, so a configuration error ends the run here.
SUBROUTINE mpi_finalize(ierror)
    INTEGER :: ierror
    WRITE (*, '(A,I0)') 'mpi_finalize called by flux_calculator_basic, code ', ierror
    ERROR STOP 2
END SUBROUTINE mpi_finalize

! The coupled host's abort routine (test stand-in for one that calls oasis_abort(comp_id,
! comp_name, msg), flux_calculator.F90:883-887): reports the message and ends the run with 3.
SUBROUTINE host_abort(msg) BIND(C)
    USE, INTRINSIC :: iso_c_binding, ONLY: c_char
    USE fcx_c_api, ONLY: fcx_c_string
    CHARACTER(kind=c_char), DIMENSION(*), INTENT(IN) :: msg
    WRITE (*, '(2A)') 'HOST ABORT ROUTINE: ', TRIM(fcx_c_string(msg))
    ERROR STOP 3
END SUBROUTINE host_abort
