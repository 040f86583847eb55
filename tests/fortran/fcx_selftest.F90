! fcx_selftest.F90 -- TEST INFRASTRUCTURE: a Fortran host driving libfcx through the
! iso_c_binding interfaces (fcx_c_api), checked against the REFERENCE flux_lib called
! directly from Fortran (compiled from /root/reference into oracle/_ref).  One CCLM and one
! MOM5 coupling step, T=1, u/v grids aliased to the t grid, bias corrections on.  A third
! step (CCLM) runs on arrays the library allocated (fcx_host_malloc + c_f_pointer: the
! default zero-copy path), with the exchange -> atmosphere accumulation, engine-owned
! boundary slots and an RCCL communicator of one rank attached (fcx_comm_*, fcx_set_comm);
! its atmosphere outputs must equal the sequential sum of its own fluxes bit for bit.
! Prints "FCX_FORTRAN_SELFTEST OK <max mixed error>" and stops 0 when every field is
! within 1e-10 (SURVEY.md 8d metric), stops 1 otherwise.
PROGRAM fcx_selftest
  USE, INTRINSIC :: iso_c_binding
  USE fcx_c_api
  USE flux_library
  IMPLICIT NONE
  INTEGER, PARAMETER :: n = 10001, dp = c_double
  INTEGER, PARAMETER :: ALBE=1, AMOI=3, AMOM=4, FICE=6, PATM=7, PSUR=8, QATM=9, TATM=10, TSUR=11, &
                        UATM=12, VATM=13, CMOM=16, CMOI=17, CHEA=18, QSUR=19, HLAT=20, HSEN=21, &
                        MEVA=22, RBBR=26, UMOM=34, VMOM=35
  REAL(dp), TARGET :: fi(n), ps(n), ts(n), pa(n), qa(n), ta(n), u(n), v(n), ai(n), am(n), &
                      ci(n), ch(n), cm(n)
  REAL(dp), TARGET :: qs(n), me(n), hl(n), hs(n), rb(n), um(n), vm(n)
  REAL(dp), TARGET :: corr(12, n)
  REAL(dp) :: r_qs(n), r_me(n), r_hl(n), r_hs(n), r_rb(n), r_um(n), r_vm(n), dummy, worst
  INTEGER :: j, variant, month
  INTEGER(c_int32_t) :: t_step, m32
  TYPE(c_ptr) :: eng
  CHARACTER(len=4) :: vname
  ! part 3: library arrays, atmosphere accumulation, communicator
  INTEGER, PARAMETER :: na = (n + 3) / 4, nfa = 4
  TYPE(c_ptr) :: comm, blk(nfa + 7)
  INTEGER(c_int8_t) :: uid(FCX_COMM_ID_BYTES)
  INTEGER(c_int32_t), TARGET :: aidx(n)
  REAL(dp), TARGET :: aw(n)
  REAL(dp), POINTER :: lme(:), lhl(:), lhs(:), lrb(:), lqs(:), lum(:), lvm(:)
  REAL(dp), POINTER :: ao(:, :)
  REAL(dp) :: want(na)
  INTEGER(c_int64_t) :: zc
  INTEGER :: k, f

  DO j = 1, n   ! deterministic inputs in the ranges of SURVEY.md 8d
    fi(j) = MERGE(1.0_dp, 0.0_dp, MOD(j, 5) == 0)
    ts(j) = MERGE(255.0_dp + 18.0_dp * ABS(SIN(0.37_dp * j)), 271.0_dp + 32.0_dp * ABS(SIN(0.11_dp * j)), fi(j) == 1.0_dp)
    ps(j) = 95000.0_dp + 10000.0_dp * ABS(COS(0.013_dp * j))
    pa(j) = ps(j) - 50.0_dp - 1450.0_dp * ABS(SIN(0.07_dp * j))
    ta(j) = ts(j) + 3.0_dp * SIN(1.3_dp * j)
    qa(j) = 5.0e-4_dp + 1.95e-2_dp * ABS(SIN(0.21_dp * j))
    u(j) = 9.0_dp * SIN(0.017_dp * j)
    v(j) = 9.0_dp * COS(0.023_dp * j)
    IF (MOD(j, 97) == 0) THEN
      u(j) = 11.0_dp; v(j) = 0.0_dp
    END IF
    ai(j) = 5.0e-4_dp + 2.5e-3_dp * ABS(SIN(0.31_dp * j)); am(j) = 5.0e-4_dp + 2.5e-3_dp * ABS(COS(0.29_dp * j))
    ci(j) = 8.0e-4_dp + 1.7e-3_dp * ABS(SIN(0.41_dp * j)); ch(j) = 8.0e-4_dp + 1.7e-3_dp * ABS(COS(0.43_dp * j))
    cm(j) = 8.0e-4_dp + 1.7e-3_dp * ABS(SIN(0.47_dp * j))
    corr(:, j) = 1.0e-5_dp * SIN(0.5_dp * j + [(REAL(month, dp), month = 1, 12)])
  END DO
  t_step = 3600 * 24 * 40   ! 1961-02-10: February slice
  CALL chk(fcx_current_month(19610101_c_int32_t, INT(t_step, c_int64_t), m32), 'month')
  month = m32

  worst = 0.0_dp
  DO variant = 1, 2
    vname = MERGE('CCLM', 'MOM5', variant == 1)
    qs = -1.0_dp; me = -1.0_dp; hl = -1.0_dp; hs = -1.0_dp; rb = -1.0_dp; um = -1.0_dp; vm = -1.0_dp
    CALL chk(fcx_create(0_c_int, 1_c_int, [INT(n, c_int32_t), INT(n, c_int32_t), INT(n, c_int32_t)], eng), 'create')
    CALL chk(fcx_set_method(eng, FCX_SPEC_VAPOR_SURFACE_T, 1_c_int, fcx_method_id('CCLM')), 'm')
    CALL chk(fcx_set_method(eng, FCX_SPEC_VAPOR_SURFACE_U, 1_c_int, fcx_method_id('CCLM')), 'm')
    CALL chk(fcx_set_method(eng, FCX_SPEC_VAPOR_SURFACE_V, 1_c_int, fcx_method_id('CCLM')), 'm')
    CALL chk(fcx_set_method(eng, FCX_FLUX_MASS_EVAP, 1_c_int, fcx_method_id(vname)), 'm')
    CALL chk(fcx_set_method(eng, FCX_FLUX_HEAT_LATENT, 1_c_int, fcx_method_id('water')), 'm')
    CALL chk(fcx_set_method(eng, FCX_FLUX_HEAT_SENSIBLE, 1_c_int, fcx_method_id(vname)), 'm')
    CALL chk(fcx_set_method(eng, FCX_FLUX_MOMENTUM, 1_c_int, fcx_method_id(vname)), 'm')
    CALL chk(fcx_set_method(eng, FCX_FLUX_RADIATION_BLACKBODY, 1_c_int, fcx_method_id('StBo')), 'm')
    CALL bind_all(1); CALL bind_all(2); CALL bind_all(3)
    CALL chk(fcx_bind_field(eng, 1_c_int, 2_c_int, UMOM, c_loc(um), INT(n, c_int64_t), FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, 3_c_int, VMOM, c_loc(vm), INT(n, c_int64_t), FCX_ALLOCATED), 'b')
    CALL chk(fcx_set_corrections(eng, 1_c_int, 19610101_c_int32_t, c_loc(corr), INT(n, c_int64_t), &
                                 FCX_CORR_CELL_MAJOR), 'corr')
    CALL chk(fcx_commit(eng), 'commit')
    CALL chk(fcx_step(eng, FCX_PHASE_ALL, t_step), 'step')
    CALL chk(fcx_destroy(eng), 'destroy')

    ! the reference, in the order of flux_calculator.F90:902-991 (calc:25-345 bindings)
    DO j = 1, n
      CALL flux_radiation_blackbody_StBo(r_rb(j), ts(j))
      CALL spec_vapor_surface_cclm(r_qs(j), fi(j), ps(j), ts(j))
      IF (variant == 1) THEN
        CALL flux_mass_evap_cclm(r_me(j), ai(j), ps(j), qa(j), r_qs(j), ta(j), u(j), v(j))
      ELSE
        CALL flux_mass_evap_mom5(r_me(j), ci(j), ps(j), qa(j), r_qs(j), ta(j), u(j), v(j))
      END IF
      r_me(j) = r_me(j) + corr(month, j)
      CALL flux_heat_latent_water(r_hl(j), r_me(j))
      IF (variant == 1) THEN
        CALL flux_heat_sensible_cclm(r_hs(j), ai(j), pa(j), ps(j), qa(j), ta(j), ts(j), u(j), v(j))
        CALL flux_momentum_cclm(r_um(j), dummy, am(j), ps(j), r_qs(j), ts(j), u(j), v(j))
        CALL flux_momentum_cclm(dummy, r_vm(j), am(j), ps(j), r_qs(j), ts(j), u(j), v(j))
      ELSE
        CALL flux_heat_sensible_mom5(r_hs(j), ch(j), pa(j), ps(j), qa(j), ta(j), ts(j), u(j), v(j))
        CALL flux_momentum_mom5(r_um(j), dummy, cm(j), ps(j), r_qs(j), ts(j), u(j), v(j))
        CALL flux_momentum_mom5(dummy, r_vm(j), cm(j), ps(j), r_qs(j), ts(j), u(j), v(j))
      END IF
    END DO
    worst = MAX(worst, err(qs, r_qs), err(me, r_me), err(hl, r_hl), err(hs, r_hs), err(rb, r_rb), &
                err(um, r_um), err(vm, r_vm))
    WRITE (*, '(A,A,A,ES12.4)') 'variant ', vname, ' max mixed error ', worst
  END DO
  ! ---- part 3 (CCLM again): outputs in library memory, accumulation, communicator
  DO j = 1, n   ! 4 exchange cells per atmosphere cell, weights summing to 1
    aidx(j) = INT((j - 1) / 4, c_int32_t)
    aw(j) = 0.25_dp
  END DO
  CALL chk(fcx_host_malloc(INT(8 * n, c_size_t), blk(1)), 'host_malloc'); CALL c_f_pointer(blk(1), lme, [n])
  CALL chk(fcx_host_malloc(INT(8 * n, c_size_t), blk(2)), 'host_malloc'); CALL c_f_pointer(blk(2), lhl, [n])
  CALL chk(fcx_host_malloc(INT(8 * n, c_size_t), blk(3)), 'host_malloc'); CALL c_f_pointer(blk(3), lhs, [n])
  CALL chk(fcx_host_malloc(INT(8 * n, c_size_t), blk(4)), 'host_malloc'); CALL c_f_pointer(blk(4), lrb, [n])
  CALL chk(fcx_host_malloc(INT(8 * n, c_size_t), blk(5)), 'host_malloc'); CALL c_f_pointer(blk(5), lqs, [n])
  CALL chk(fcx_host_malloc(INT(8 * n, c_size_t), blk(6)), 'host_malloc'); CALL c_f_pointer(blk(6), lum, [n])
  CALL chk(fcx_host_malloc(INT(8 * n, c_size_t), blk(7)), 'host_malloc'); CALL c_f_pointer(blk(7), lvm, [n])
  CALL chk(fcx_host_malloc(INT(8 * na * nfa, c_size_t), blk(8)), 'host_malloc'); CALL c_f_pointer(blk(8), ao, [na, nfa])
  lme = -1.0_dp; lhl = -1.0_dp; lhs = -1.0_dp; lrb = -1.0_dp; lqs = -1.0_dp; lum = -1.0_dp; lvm = -1.0_dp
  ao = -1.0_dp
  CALL chk(fcx_comm_unique_id(uid), 'unique id')   ! rank 0; an MPI host broadcasts it
  CALL chk(fcx_comm_create(0_c_int, 1_c_int, 0_c_int, uid, comm), 'comm create')
  CALL chk(fcx_create(0_c_int, 1_c_int, [INT(n, c_int32_t), INT(n, c_int32_t), INT(n, c_int32_t)], eng), 'create')
  CALL chk(fcx_set_method(eng, FCX_SPEC_VAPOR_SURFACE_T, 1_c_int, fcx_method_id('CCLM')), 'm')
  CALL chk(fcx_set_method(eng, FCX_SPEC_VAPOR_SURFACE_U, 1_c_int, fcx_method_id('CCLM')), 'm')
  CALL chk(fcx_set_method(eng, FCX_SPEC_VAPOR_SURFACE_V, 1_c_int, fcx_method_id('CCLM')), 'm')
  CALL chk(fcx_set_method(eng, FCX_FLUX_MASS_EVAP, 1_c_int, fcx_method_id('CCLM')), 'm')
  CALL chk(fcx_set_method(eng, FCX_FLUX_HEAT_LATENT, 1_c_int, fcx_method_id('water')), 'm')
  CALL chk(fcx_set_method(eng, FCX_FLUX_HEAT_SENSIBLE, 1_c_int, fcx_method_id('CCLM')), 'm')
  CALL chk(fcx_set_method(eng, FCX_FLUX_MOMENTUM, 1_c_int, fcx_method_id('CCLM')), 'm')
  CALL chk(fcx_set_method(eng, FCX_FLUX_RADIATION_BLACKBODY, 1_c_int, fcx_method_id('StBo')), 'm')
  CALL bind_inputs(1); CALL bind_inputs(2); CALL bind_inputs(3)
  DO k = 1, 3   ! the u/v grids alias the t-grid arrays
    CALL chk(fcx_bind_field(eng, 1_c_int, INT(k, c_int), QSUR, c_loc(lqs), INT(n, c_int64_t), FCX_ALLOCATED), 'b')
  END DO
  CALL chk(fcx_bind_field(eng, 1_c_int, 1_c_int, MEVA, c_loc(lme), INT(n, c_int64_t), FCX_ALLOCATED), 'b')
  CALL chk(fcx_bind_field(eng, 1_c_int, 1_c_int, HLAT, c_loc(lhl), INT(n, c_int64_t), FCX_ALLOCATED), 'b')
  CALL chk(fcx_bind_field(eng, 1_c_int, 1_c_int, HSEN, c_loc(lhs), INT(n, c_int64_t), FCX_ALLOCATED), 'b')
  CALL chk(fcx_bind_field(eng, 1_c_int, 1_c_int, RBBR, c_loc(lrb), INT(n, c_int64_t), FCX_ALLOCATED), 'b')
  CALL chk(fcx_bind_field(eng, 1_c_int, 2_c_int, UMOM, c_loc(lum), INT(n, c_int64_t), FCX_ALLOCATED), 'b')
  CALL chk(fcx_bind_field(eng, 1_c_int, 3_c_int, VMOM, c_loc(lvm), INT(n, c_int64_t), FCX_ALLOCATED), 'b')
  CALL chk(fcx_set_corrections(eng, 1_c_int, 19610101_c_int32_t, c_loc(corr), INT(n, c_int64_t), &
                               FCX_CORR_CELL_MAJOR), 'corr')
  CALL chk(fcx_set_atmos_map(eng, INT(na, c_int64_t), c_loc(aidx), c_loc(aw)), 'atmos map')
  CALL chk(fcx_add_atmos_field(eng, FCX_PHASE_NORMAL, 1_c_int, 1_c_int, MEVA, c_loc(ao(1, 1)), FCX_MEM_HOST), 'af')
  CALL chk(fcx_add_atmos_field(eng, FCX_PHASE_NORMAL, 1_c_int, 1_c_int, HLAT, c_loc(ao(1, 2)), FCX_MEM_HOST), 'af')
  CALL chk(fcx_add_atmos_field(eng, FCX_PHASE_NORMAL, 1_c_int, 1_c_int, HSEN, c_loc(ao(1, 3)), FCX_MEM_HOST), 'af')
  CALL chk(fcx_add_atmos_field(eng, FCX_PHASE_NORMAL, 1_c_int, 2_c_int, UMOM, c_loc(ao(1, 4)), FCX_MEM_HOST), 'af')
  ! one boundary slot for the last atmosphere cell (with one rank the all-reduce is the
  ! identity, so the completed value is the full sum)
  CALL chk(fcx_set_atmos_boundaries(eng, 1_c_int32_t, -1_c_int32_t, 0_c_int32_t), 'boundaries')
  CALL chk(fcx_set_comm(eng, comm), 'set comm')
  CALL chk(fcx_commit(eng), 'commit')
  CALL chk(fcx_zero_copy_bytes(eng, zc), 'zero copy bytes')
  IF (zc <= 0) THEN
    WRITE (*, *) 'library arrays were not used in place'
    STOP 1
  END IF
  CALL chk(fcx_step(eng, FCX_PHASE_ALL, t_step), 'step')
  CALL chk(fcx_destroy(eng), 'destroy')
  CALL chk(fcx_comm_destroy(comm), 'comm destroy')
  DO j = 1, n   ! CCLM reference again
    CALL flux_radiation_blackbody_StBo(r_rb(j), ts(j))
    CALL spec_vapor_surface_cclm(r_qs(j), fi(j), ps(j), ts(j))
    CALL flux_mass_evap_cclm(r_me(j), ai(j), ps(j), qa(j), r_qs(j), ta(j), u(j), v(j))
    r_me(j) = r_me(j) + corr(month, j)
    CALL flux_heat_latent_water(r_hl(j), r_me(j))
    CALL flux_heat_sensible_cclm(r_hs(j), ai(j), pa(j), ps(j), qa(j), ta(j), ts(j), u(j), v(j))
    CALL flux_momentum_cclm(r_um(j), dummy, am(j), ps(j), r_qs(j), ts(j), u(j), v(j))
    CALL flux_momentum_cclm(dummy, r_vm(j), am(j), ps(j), r_qs(j), ts(j), u(j), v(j))
  END DO
  worst = MAX(worst, err(lqs, r_qs), err(lme, r_me), err(lhl, r_hl), err(lhs, r_hs), err(lrb, r_rb), &
              err(lum, r_um), err(lvm, r_vm))
  WRITE (*, '(A,ES12.4)') 'library arrays + accumulation + comm, max mixed error ', worst
  DO f = 1, nfa   ! sequential SCRIP sums of the engine's own fluxes, increasing exchange cell
    want = 0.0_dp
    DO j = 1, n
      SELECT CASE (f)
      CASE (1); want(aidx(j) + 1) = want(aidx(j) + 1) + aw(j) * lme(j)
      CASE (2); want(aidx(j) + 1) = want(aidx(j) + 1) + aw(j) * lhl(j)
      CASE (3); want(aidx(j) + 1) = want(aidx(j) + 1) + aw(j) * lhs(j)
      CASE (4); want(aidx(j) + 1) = want(aidx(j) + 1) + aw(j) * lum(j)
      END SELECT
    END DO
    IF (ANY(ao(:, f) /= want)) THEN
      WRITE (*, *) 'atmosphere field ', f, ' differs from the sequential sum: ', COUNT(ao(:, f) /= want), ' cells'
      STOP 1
    END IF
  END DO
  DO k = 1, 8
    CALL chk(fcx_host_free(blk(k)), 'host_free')
  END DO

  IF (worst <= 1.0e-10_dp) THEN
    WRITE (*, '(A,ES12.4)') 'FCX_FORTRAN_SELFTEST OK ', worst
  ELSE
    WRITE (*, '(A,ES12.4)') 'FCX_FORTRAN_SELFTEST FAIL ', worst
    STOP 1
  END IF

CONTAINS

  SUBROUTINE chk(status, what)
    INTEGER(c_int), INTENT(IN) :: status
    CHARACTER(len=*), INTENT(IN) :: what
    IF (status /= FCX_OK) THEN
      WRITE (*, *) 'fcx error in ', what, ': ', TRIM(fcx_error_message())
      STOP 1
    END IF
  END SUBROUTINE

  SUBROUTINE bind_all(g)   ! the u/v grids alias the t-grid arrays (same addresses)
    INTEGER, INTENT(IN) :: g
    INTEGER(c_int) :: gg
    INTEGER(c_int64_t) :: nn
    gg = INT(g, c_int); nn = INT(n, c_int64_t)
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, FICE, c_loc(fi), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, PSUR, c_loc(ps), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, TSUR, c_loc(ts), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, PATM, c_loc(pa), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, QATM, c_loc(qa), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, TATM, c_loc(ta), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, UATM, c_loc(u), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, VATM, c_loc(v), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, AMOI, c_loc(ai), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, AMOM, c_loc(am), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, CMOI, c_loc(ci), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, CHEA, c_loc(ch), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, CMOM, c_loc(cm), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, QSUR, c_loc(qs), nn, FCX_ALLOCATED), 'b')
    IF (g == 1) THEN
      CALL chk(fcx_bind_field(eng, 1_c_int, gg, MEVA, c_loc(me), nn, FCX_ALLOCATED), 'b')
      CALL chk(fcx_bind_field(eng, 1_c_int, gg, HLAT, c_loc(hl), nn, FCX_ALLOCATED), 'b')
      CALL chk(fcx_bind_field(eng, 1_c_int, gg, HSEN, c_loc(hs), nn, FCX_ALLOCATED), 'b')
      CALL chk(fcx_bind_field(eng, 1_c_int, gg, RBBR, c_loc(rb), nn, FCX_ALLOCATED), 'b')
    END IF
  END SUBROUTINE

  SUBROUTINE bind_inputs(g)   ! the t-grid inputs under every grid (aliases)
    INTEGER, INTENT(IN) :: g
    INTEGER(c_int) :: gg
    INTEGER(c_int64_t) :: nn
    gg = INT(g, c_int); nn = INT(n, c_int64_t)
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, FICE, c_loc(fi), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, PSUR, c_loc(ps), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, TSUR, c_loc(ts), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, PATM, c_loc(pa), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, QATM, c_loc(qa), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, TATM, c_loc(ta), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, UATM, c_loc(u), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, VATM, c_loc(v), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, AMOI, c_loc(ai), nn, FCX_ALLOCATED), 'b')
    CALL chk(fcx_bind_field(eng, 1_c_int, gg, AMOM, c_loc(am), nn, FCX_ALLOCATED), 'b')
  END SUBROUTINE

  FUNCTION err(x, r) RESULT(e)   ! SURVEY.md 8d mixed metric
    REAL(dp), INTENT(IN) :: x(:), r(:)
    REAL(dp) :: e, scale
    INTEGER :: k
    e = 0.0_dp
    DO k = 1, SIZE(r)
      scale = MAX(ABS(r(k)), 1.0e-6_dp * MAXVAL(ABS(r)))
      e = MAX(e, ABS(x(k) - r(k)) / scale)
    END DO
  END FUNCTION

END PROGRAM fcx_selftest
