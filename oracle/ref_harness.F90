! ref_harness.F90 -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
!
! Drives the REFERENCE flux_lib (compiled unmodified from /root/reference/src/flux_lib by
! oracle/Makefile, with the production -r8 semantics: -fdefault-real-8) over the oracle
! state struct of oracle/fco.h.  The loops below restate flux_calculator_calculate.F90
! (calc:25-385): that module itself cannot be built here because it USEs
! bias_corrections (needs the absent NetCDF-Fortran module) and call_python (needs the
! cffi-generated libpyfort), so its ~60 lines of loop/dispatch glue are restated and every
! per-cell result comes from the reference flux_lib routines themselves.
!
! Never linked into the product.  Used by tests/golden/make_golden.py (fixture
! generation), by tests (live cross-check when oracle/_ref is built) and by bench.py's
! cpu_baseline leg (kind "reference").
module fco_ref_harness
  use, intrinsic :: iso_c_binding
  use flux_library
  implicit none
  private

  integer, parameter :: NV = 35, MT = 10, NF = 8
  ! var ids (flux_calculator_basic.F90:43-51), 1-based
  integer, parameter :: IDX_AMOI = 3, IDX_AMOM = 4, IDX_FARE = 5, IDX_FICE = 6, IDX_PATM = 7, &
                        IDX_PSUR = 8, IDX_QATM = 9, IDX_TATM = 10, IDX_TSUR = 11, IDX_UATM = 12, &
                        IDX_VATM = 13, IDX_CMOM = 16, IDX_CMOI = 17, IDX_CHEA = 18, IDX_QSUR = 19, &
                        IDX_HLAT = 20, IDX_HSEN = 21, IDX_MEVA = 22, IDX_RBBR = 26, IDX_RSDD = 32, &
                        IDX_RSDR = 33, IDX_UMOM = 34, IDX_VMOM = 35
  integer, parameter :: M_NONE = 0, M_ZERO = 1, M_COPY = 2, M_CCLM = 3, M_MOM5 = 4, M_RCO = 5, &
                        M_WATER = 6, M_ICE = 7, M_STBO = 8
  integer, parameter :: F_QSUR_T = 1, F_MEVA = 4, F_HLAT = 5, F_HSEN = 6, F_MOM = 7, F_RBBR = 8

  type, bind(c) :: fco_matrix
    integer(c_int32_t) :: num_elements, pad
    type(c_ptr) :: src_index, dst_index, weight
  end type

  type, bind(c) :: fco_state
    integer(c_int32_t) :: num_surface_types
    integer(c_int32_t) :: grid_size(3)
    integer(c_int32_t) :: method(MT, NF)
    integer(c_int32_t) :: lcorrections, current_month
    type(c_ptr) :: corrections
    type(c_ptr) :: field(NV, 3, 0:MT)
    integer(c_int8_t) :: allocated(NV, 3, 0:MT)
    integer(c_int8_t) :: put_to(NV, 3, 0:MT)
    type(fco_matrix) :: regrid(4)
  end type

  public :: fco_state

contains

  function fld(st, s, g, v) result(p)
    type(fco_state), intent(in) :: st
    integer, intent(in) :: s, g, v
    real(c_double), pointer :: p(:)
    call c_f_pointer(st%field(v, g, s), p, [max(st%grid_size(g), 1)])
  end function

  ! calc:25-50
  subroutine ref_calc_spec_vapor_surface(st, g) bind(c, name='ref_calc_spec_vapor_surface')
    type(fco_state), intent(inout) :: st
    integer(c_int), value :: g
    integer :: i, j
    real(c_double), pointer :: q(:), fi(:), ps(:), ts(:)
    do i = 1, st%num_surface_types
      if (st%method(i, F_QSUR_T + g - 1) == M_CCLM) then
        q => fld(st, i, g, IDX_QSUR); fi => fld(st, i, g, IDX_FICE)
        ps => fld(st, i, g, IDX_PSUR); ts => fld(st, i, g, IDX_TSUR)
        do j = 1, st%grid_size(g)
          call spec_vapor_surface_cclm(q(j), fi(j), ps(j), ts(j))
        end do
      end if
    end do
  end subroutine

  ! calc:54-120
  subroutine ref_calc_flux_mass_evap(st) bind(c, name='ref_calc_flux_mass_evap')
    type(fco_state), intent(inout) :: st
    integer :: i, j, m, n
    real(c_double), pointer :: o(:), a(:), ps(:), qa(:), qs(:), ta(:), ts(:), u(:), v(:)
    real(c_double), pointer :: corr(:, :, :)
    n = st%grid_size(1)
    do i = 1, st%num_surface_types
      m = st%method(i, F_MEVA)
      if (m == M_NONE) cycle
      o => fld(st, i, 1, IDX_MEVA)
      if (m == M_ZERO) then
        o(1:n) = 0.0
      else if (m == M_CCLM .or. m == M_MOM5) then
        if (m == M_CCLM) then
          a => fld(st, i, 1, IDX_AMOI)
        else
          a => fld(st, i, 1, IDX_CMOI)
        end if
        ps => fld(st, i, 1, IDX_PSUR); qa => fld(st, i, 1, IDX_QATM); qs => fld(st, i, 1, IDX_QSUR)
        ta => fld(st, i, 1, IDX_TATM); u => fld(st, i, 1, IDX_UATM); v => fld(st, i, 1, IDX_VATM)
        do j = 1, n
          if (m == M_CCLM) then
            call flux_mass_evap_cclm(o(j), a(j), ps(j), qa(j), qs(j), ta(j), u(j), v(j))
          else
            call flux_mass_evap_mom5(o(j), a(j), ps(j), qa(j), qs(j), ta(j), u(j), v(j))
          end if
        end do
      else if (m == M_RCO) then
        qa => fld(st, i, 1, IDX_QATM); ts => fld(st, i, 1, IDX_TSUR)
        u => fld(st, i, 1, IDX_UATM); v => fld(st, i, 1, IDX_VATM)
        do j = 1, n
          call flux_mass_evap_rco(o(j), qa(j), ts(j), u(j), v(j))
        end do
      end if
      if (st%lcorrections /= 0) then
        call c_f_pointer(st%corrections, corr, [1, 12, max(n, 1)])
        do j = 1, n
          o(j) = o(j) + corr(1, st%current_month, j)
        end do
      end if
    end do
  end subroutine

  ! calc:124-154
  subroutine ref_calc_flux_heat_latent(st) bind(c, name='ref_calc_flux_heat_latent')
    type(fco_state), intent(inout) :: st
    integer :: i, j, m, n
    real(c_double), pointer :: o(:), e(:)
    n = st%grid_size(1)
    do i = 1, st%num_surface_types
      m = st%method(i, F_HLAT)
      if (m == M_NONE) cycle
      o => fld(st, i, 1, IDX_HLAT)
      if (m == M_ZERO) then
        o(1:n) = 0.0
      else if (m == M_WATER) then
        e => fld(st, i, 1, IDX_MEVA)
        do j = 1, n
          call flux_heat_latent_water(o(j), e(j))
        end do
      else if (m == M_ICE) then
        e => fld(st, i, 1, IDX_MEVA)
        do j = 1, n
          call flux_heat_latent_ice(o(j), e(j))
        end do
      end if
    end do
  end subroutine

  ! calc:156-208
  subroutine ref_calc_flux_heat_sensible(st) bind(c, name='ref_calc_flux_heat_sensible')
    type(fco_state), intent(inout) :: st
    integer :: i, j, m, n
    real(c_double), pointer :: o(:), a(:), pa(:), ps(:), qa(:), ta(:), ts(:), u(:), v(:)
    n = st%grid_size(1)
    do i = 1, st%num_surface_types
      m = st%method(i, F_HSEN)
      if (m == M_NONE) cycle
      o => fld(st, i, 1, IDX_HSEN)
      if (m == M_ZERO) then
        o(1:n) = 0.0
        cycle
      end if
      ta => fld(st, i, 1, IDX_TATM); ts => fld(st, i, 1, IDX_TSUR)
      u => fld(st, i, 1, IDX_UATM); v => fld(st, i, 1, IDX_VATM)
      if (m == M_CCLM .or. m == M_MOM5) then
        if (m == M_CCLM) then
          a => fld(st, i, 1, IDX_AMOI)
        else
          a => fld(st, i, 1, IDX_CHEA)
        end if
        pa => fld(st, i, 1, IDX_PATM); ps => fld(st, i, 1, IDX_PSUR); qa => fld(st, i, 1, IDX_QATM)
        do j = 1, n
          if (m == M_CCLM) then
            call flux_heat_sensible_cclm(o(j), a(j), pa(j), ps(j), qa(j), ta(j), ts(j), u(j), v(j))
          else
            call flux_heat_sensible_mom5(o(j), a(j), pa(j), ps(j), qa(j), ta(j), ts(j), u(j), v(j))
          end if
        end do
      else if (m == M_RCO) then
        do j = 1, n
          call flux_heat_sensible_rco(o(j), ta(j), ts(j), u(j), v(j))
        end do
      end if
    end do
  end subroutine

  ! calc:212-316 (north = 0 -> east component kept, 1 -> north component kept)
  subroutine momentum(st, g, north)
    type(fco_state), intent(inout) :: st
    integer, intent(in) :: g, north
    integer :: i, j, m, n, var
    real(c_double) :: dummy
    real(c_double), pointer :: o(:), a(:), ps(:), qs(:), ts(:), u(:), v(:)
    n = st%grid_size(g)
    var = IDX_UMOM
    if (north /= 0) var = IDX_VMOM
    do i = 1, st%num_surface_types
      m = st%method(i, F_MOM)
      if (m == M_NONE) cycle
      o => fld(st, i, g, var)
      if (m == M_ZERO) then
        o(1:n) = 0.0
        cycle
      end if
      u => fld(st, i, g, IDX_UATM); v => fld(st, i, g, IDX_VATM)
      if (m == M_CCLM .or. m == M_MOM5) then
        if (m == M_CCLM) then
          a => fld(st, i, g, IDX_AMOM)
        else
          a => fld(st, i, g, IDX_CMOM)
        end if
        ps => fld(st, i, g, IDX_PSUR); qs => fld(st, i, g, IDX_QSUR); ts => fld(st, i, g, IDX_TSUR)
        do j = 1, n
          if (north == 0) then
            if (m == M_CCLM) then
              call flux_momentum_cclm(o(j), dummy, a(j), ps(j), qs(j), ts(j), u(j), v(j))
            else
              call flux_momentum_mom5(o(j), dummy, a(j), ps(j), qs(j), ts(j), u(j), v(j))
            end if
          else
            if (m == M_CCLM) then
              call flux_momentum_cclm(dummy, o(j), a(j), ps(j), qs(j), ts(j), u(j), v(j))
            else
              call flux_momentum_mom5(dummy, o(j), a(j), ps(j), qs(j), ts(j), u(j), v(j))
            end if
          end if
        end do
      else if (m == M_RCO) then
        do j = 1, n
          if (north == 0) then
            call flux_momentum_rco(o(j), dummy, u(j), v(j))
          else
            call flux_momentum_rco(dummy, o(j), u(j), v(j))
          end if
        end do
      end if
    end do
  end subroutine

  subroutine ref_calc_flux_momentum_east(st, g) bind(c, name='ref_calc_flux_momentum_east')
    type(fco_state), intent(inout) :: st
    integer(c_int), value :: g
    call momentum(st, int(g), 0)
  end subroutine

  subroutine ref_calc_flux_momentum_north(st, g) bind(c, name='ref_calc_flux_momentum_north')
    type(fco_state), intent(inout) :: st
    integer(c_int), value :: g
    call momentum(st, int(g), 1)
  end subroutine

  ! calc:320-345
  subroutine ref_calc_flux_radiation_blackbody(st) bind(c, name='ref_calc_flux_radiation_blackbody')
    type(fco_state), intent(inout) :: st
    integer :: i, j, m, n
    real(c_double), pointer :: o(:), ts(:)
    n = st%grid_size(1)
    do i = 1, st%num_surface_types
      m = st%method(i, F_RBBR)
      if (m == M_NONE) cycle
      o => fld(st, i, 1, IDX_RBBR)
      if (m == M_ZERO) then
        o(1:n) = 0.0
      else if (m == M_STBO) then
        ts => fld(st, i, 1, IDX_TSUR)
        do j = 1, n
          call flux_radiation_blackbody_StBo(o(j), ts(j))
        end do
      end if
    end do
  end subroutine

  ! calc:347-364 (skipped when RSDD/RSDR are not associated, P6)
  subroutine ref_distribute_shortwave_radiation_flux(st) bind(c, name='ref_distribute_shortwave_radiation_flux')
    type(fco_state), intent(inout) :: st
    integer :: i, j, n
    real(c_double), pointer :: o(:), rsdd(:), alba(:), albe(:)
    real(c_double), target :: zero1(1)
    n = st%grid_size(1)
    if (.not. c_associated(st%field(IDX_RSDD, 1, 0))) return
    zero1 = 0.0
    rsdd => fld(st, 0, 1, IDX_RSDD)
    alba => zero1
    if (c_associated(st%field(2, 1, 0))) alba => fld(st, 0, 1, 2)
    do i = 1, st%num_surface_types
      if (.not. c_associated(st%field(IDX_RSDR, 1, i))) return
      o => fld(st, i, 1, IDX_RSDR)
      albe => zero1
      if (c_associated(st%field(1, 1, i))) albe => fld(st, i, 1, 1)
      do j = 1, n
        call distribute_radiation_flux(o(j), rsdd(j), alba(min(j, size(alba))), albe(min(j, size(albe))))
      end do
    end do
  end subroutine

  ! calc:368-385
  subroutine ref_average_across_surface_types(st, g, var) bind(c, name='ref_average_across_surface_types')
    type(fco_state), intent(inout) :: st
    integer(c_int), value :: g, var
    integer :: i, j, n
    real(c_double), pointer :: x0(:), x(:), fa(:)
    if (st%allocated(var + 1, g, 0) == 0) return
    n = st%grid_size(g)
    x0 => fld(st, 0, g, var + 1)
    x0(1:n) = 0.0
    do i = 1, st%num_surface_types
      x => fld(st, i, g, var + 1); fa => fld(st, i, g, IDX_FARE)
      do j = 1, n
        x0(j) = x0(j) + x(j) * fa(j)
      end do
    end do
  end subroutine

end module fco_ref_harness
