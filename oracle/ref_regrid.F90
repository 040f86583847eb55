! ref_regrid.F90 -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
!
! Calls the REFERENCE do_regridding (flux_calculator_basic.F90:463-522), compiled unmodified
! from /root/reference/src/flux_calculator_basic.F90 by oracle/Makefile (target basic-mod),
! over the oracle state struct of oracle/fco.h: the state's field pointers, allocated and
! put_to flags become a local_field(0:MAX_SURFACE_TYPES, 3) of the reference's own
! local_fields_type (pointer association, no copies), its four COO matrices become the
! reference's sparse_regridding_matrix values, and the reference routine does the work.
! This pins oracle/fco.c:fco_do_regridding and, through it, libfcx's regrid_csr_kernel.
!
! Never linked into the product.  Used by tests/golden/make_golden.py and by the live
! cross-check in tests/test_oracle_golden.py when oracle/_ref is built.
module fco_ref_regrid
  use, intrinsic :: iso_c_binding
  use flux_calculator_basic, only: local_fields_type, sparse_regridding_matrix, do_regridding, &
                                   nullify_localvars, MAX_SURFACE_TYPES, MAX_VARNAMES
  implicit none
  private

  integer, parameter :: NV = 35, MT = 10, NF = 8

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

contains

  subroutine to_matrix(c, m)
    type(fco_matrix), intent(in) :: c
    type(sparse_regridding_matrix), intent(out) :: m
    integer(c_int32_t), pointer :: si(:), di(:)
    real(c_double), pointer :: w(:)
    m%num_elements = c%num_elements
    nullify(m%src_index%field, m%dst_index%field, m%weight%field)
    m%src_index%allocated = .false.
    m%dst_index%allocated = .false.
    m%weight%allocated = .false.
    m%weight%put_to_t_grid = .false.
    m%weight%put_to_u_grid = .false.
    m%weight%put_to_v_grid = .false.
    if (c%num_elements > 0) then
      call c_f_pointer(c%src_index, si, [c%num_elements])
      call c_f_pointer(c%dst_index, di, [c%num_elements])
      call c_f_pointer(c%weight, w, [c%num_elements])
      m%src_index%field => si
      m%dst_index%field => di
      m%weight%field => w
    end if
  end subroutine

  ! do_regridding(varidx, surface_type, local_field, u_to_t, v_to_t, t_to_u, t_to_v)
  subroutine ref_do_regridding(st, var, surface_type) bind(c, name='ref_do_regridding')
    type(fco_state), intent(inout) :: st
    integer(c_int), value :: var, surface_type
    type(local_fields_type), allocatable :: lf(:, :)
    type(sparse_regridding_matrix) :: m(4)
    real(c_double), pointer :: p(:)
    integer :: s, g, v
    allocate(lf(0:MAX_SURFACE_TYPES, 3))
    do s = 0, MAX_SURFACE_TYPES
      do g = 1, 3
        call nullify_localvars(lf(s, g))
        if (s > MT) cycle
        do v = 1, min(NV, MAX_VARNAMES)
          if (c_associated(st%field(v, g, s))) then
            call c_f_pointer(st%field(v, g, s), p, [max(st%grid_size(g), 1)])
            lf(s, g)%var(v)%field => p(1:st%grid_size(g))
          end if
          lf(s, g)%var(v)%allocated = st%allocated(v, g, s) /= 0
          lf(s, g)%var(v)%put_to_t_grid = iand(int(st%put_to(v, g, s)), 1) /= 0
          lf(s, g)%var(v)%put_to_u_grid = iand(int(st%put_to(v, g, s)), 2) /= 0
          lf(s, g)%var(v)%put_to_v_grid = iand(int(st%put_to(v, g, s)), 4) /= 0
        end do
      end do
    end do
    do g = 1, 4
      call to_matrix(st%regrid(g), m(g))
    end do
    call do_regridding(int(var), int(surface_type), lf, m(1), m(2), m(3), m(4))
    deallocate(lf)
  end subroutine

end module fco_ref_regrid

! The host program's MPI finalisation: flux_calculator_basic calls mpi_finalize(1) on a
! fatal set-up error (never on the do_regridding path).  This test host has no MPI.
subroutine mpi_finalize(ierror)
  integer :: ierror
  write (*, '(A,I0)') 'mpi_finalize called by flux_calculator_basic, code ', ierror
  stop 1
end subroutine mpi_finalize
