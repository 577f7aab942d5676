! sitebond.f90 -- drop-in for Fortran/Square/sitebond.f and Fortran/
! Triangular/sitebond.f: sites filled to ps (seed sseed), then bonds to pb
! (seed bseed), mixed labeling and spanning test, on libperc.  With
! conductance = .true. it also computes the ConductCalc.m mixed-rule
! conductance (MATLAB/ConductCalc.m:132-165).
!
! Parameters: the reference's block (Square/sitebond.f:54-71: 50x50,
! Triangular 10x10; ps = pb = .50, sseed 143285, bseed 43716), overridable
! by an optional namelist file sitebond.nml (&sitebond_nml lattice, m, n,
! pbc, ps, pb, sseed, bseed, conductance, Va, g0, tol, itmax, device /).
! Outputs as the reference: sbsite.txt (i, s(i), c(i)) and sbbond.txt
! (b1, b2, label) (sitebond.f:468-477).  sbdebug.txt is not written.
program sitebond
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
  integer(c_int) :: lattice, m, n, pbc, sseed, bseed, itmax, device
  double precision :: ps, pb, Va, g0, tol
  logical :: conductance
  namelist /sitebond_nml/ lattice, m, n, pbc, ps, pb, sseed, bseed, conductance, Va, g0, tol, &
                          itmax, device
  integer(c_int) :: t, nb, ts, tb, i, rc, stats(4)
  integer(c_int), allocatable, target :: b1(:), b2(:), sorder(:), border(:), slabel(:), &
                                         blabel(:), csize(:)
  type(c_ptr) :: h
  type(perc_label_info) :: info
  type(perc_cond_result) :: res
  integer :: u

  lattice = PERC_LATTICE
  if (lattice == PERC_SQUARE) then
    m = 50
    n = 50
  else
    m = 10
    n = 10
  end if
  pbc = 0
  ps = 0.50d+00
  pb = 0.50d+00
  sseed = 143285
  bseed = 43716
  conductance = .false.
  Va = 1.00d+00
  g0 = 1.00d+00
  tol = 1.00d-08
  itmax = 100000
  device = 0
  if (perc_have_file('sitebond.nml')) then
    open(newunit=u, file='sitebond.nml', status='old')
    read(u, nml=sitebond_nml)
    close(u)
  end if

  t = m * n
  nb = perc_nbonds(lattice, m, n, pbc)
  allocate(b1(nb), b2(nb), sorder(t + 1), border(nb + 1), slabel(t), blabel(nb), &
           csize(t + nb + 2))
  rc = perc_bond_list(lattice, m, n, pbc, b1, b2)
  call perc_shuffled_ids(t, sseed, sorder)    ! sitebond.f:117-143
  call perc_shuffled_ids(nb, bseed, border)   ! sitebond.f:165-189
  ts = ps * t
  tb = pb * nb

  call perc_check(perc_ctx_create(device, lattice, m, n, pbc, h), 'perc_ctx_create')
  call perc_check(perc_occupy(h, PERC_SITEBOND, ts, c_loc(sorder), tb, c_loc(border)), &
                  'perc_occupy')
  call perc_check(perc_label(h, info, c_null_ptr), 'perc_label')
  call perc_check(perc_label_numbers(h, c_loc(blabel), c_loc(slabel), c_loc(csize), &
                                     t + nb + 2, stats), 'perc_label_numbers')

  write(6, *) "largest overall cluster number:", stats(2)
  write(6, *) "largest overall cluster size:", stats(3)
  if (stats(4) > 0) then
    write(6, *) "infinite cluster number:", stats(4)
  else
    write(6, *) "no infinite cluster present"
  end if
  if (conductance .and. stats(4) > 0) then
    call perc_check(perc_conductance(h, PERC_RULE_MIXED, PERC_CUR_MATLAB, Va, g0, PERC_LEAK, &
                                     2, tol, itmax, res, c_null_ptr), 'perc_conductance')
    write(6, *) "Conductance:", res%gtop, res%gbot
  end if

  open(unit=10, file='sbsite.txt')
  do i = 1, t
    write(10, 111) i, slabel(i), csize(i + 1)
  end do
  close(10)
  open(unit=11, file='sbbond.txt')
  do i = 1, nb
    write(11, 111) b1(i), b2(i), blabel(i)
  end do
  close(11)
  call perc_check(perc_ctx_destroy(h), 'perc_ctx_destroy')

111 format(i10, ",", i10, ",", i10)
end program sitebond
