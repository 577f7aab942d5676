! site.f90 -- drop-in for Fortran/Square/site.f and Fortran/Triangular/
! site.f: one site-percolation realisation filled to ps and its spanning
! test, on libperc.  With conductance = .true. (namelist) it also computes
! the ConductCalc.m site-rule conductance (MATLAB/ConductCalc.m:88-130),
! which the Fortran reference does not have.
!
! Parameters: the reference's block (Square/site.f:51-131: 50x50, ps = .60,
! seed 1080115; Triangular: ps = .548, seed 143285), overridable by an
! optional namelist file site.nml (&site_nml lattice, m, n, pbc, ps, seed,
! conductance, Va, g0, tol, itmax, device /).  Outputs as the reference:
! bondlist.txt (i10,",",i10), siteorder.txt (list-directed), site.txt
! (j, s(j), c(j); site.f:353-358).  siteocc.txt (trace) is not written.
program site
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
  integer(c_int) :: lattice, m, n, pbc, seed, itmax, device
  double precision :: ps, Va, g0, tol
  logical :: conductance
  namelist /site_nml/ lattice, m, n, pbc, ps, seed, conductance, Va, g0, tol, itmax, device
  integer(c_int) :: t, nb, tsites, i, rc, stats(4)
  integer(c_int), allocatable, target :: b1(:), b2(:), order(:), slabel(:), csize(:)
  type(c_ptr) :: h
  type(perc_label_info) :: info
  type(perc_cond_result) :: res
  integer :: u

  lattice = PERC_LATTICE
  m = 50
  n = 50
  pbc = 0
  if (lattice == PERC_SQUARE) then
    ps = 0.60d+00
    seed = 1080115
  else
    ps = 0.548d+00
    seed = 143285
  end if
  conductance = .false.
  Va = 1.00d+00
  g0 = 1.00d+00
  tol = 1.00d-08
  itmax = 100000
  device = 0
  if (perc_have_file('site.nml')) then
    open(newunit=u, file='site.nml', status='old')
    read(u, nml=site_nml)
    close(u)
  end if

  t = m * n
  nb = perc_nbonds(lattice, m, n, pbc)
  allocate(b1(nb), b2(nb), order(t + 1), slabel(t), csize(t + 2))
  rc = perc_bond_list(lattice, m, n, pbc, b1, b2)
  open(unit=13, file='bondlist.txt')
  do i = 1, nb
    write(13, 121) b1(i), b2(i)
  end do
  close(13)

  call perc_shuffled_ids(t, seed, order)
  open(unit=12, file='siteorder.txt')
  do i = 1, t
    write(12, *) order(i)
  end do
  close(12)

  tsites = ps * t
  call perc_check(perc_ctx_create(device, lattice, m, n, pbc, h), 'perc_ctx_create')
  call perc_check(perc_occupy(h, PERC_SITE, tsites, c_loc(order), 0, c_null_ptr), 'perc_occupy')
  call perc_check(perc_label(h, info, c_null_ptr), 'perc_label')
  call perc_check(perc_label_numbers(h, c_null_ptr, c_loc(slabel), c_loc(csize), t + 2, stats), &
                  'perc_label_numbers')

  write(6, *)
  write(6, *) "******************************"
  write(6, *) "largest overall cluster number:", stats(2)
  write(6, *) "largest overall cluster size:", stats(3)
  if (stats(4) > 0) then
    write(6, *) "infinite cluster present"
    write(6, *) "infinite cluster number:", stats(4)
    write(6, *) "infinite cluster size:", csize(stats(4) + 1)
  else
    write(6, *) "no infinite cluster present"
  end if
  write(6, *) "******************************"
  if (conductance .and. stats(4) > 0) then
    call perc_check(perc_conductance(h, PERC_RULE_SITE, PERC_CUR_MATLAB, Va, g0, PERC_LEAK, &
                                     2, tol, itmax, res, c_null_ptr), 'perc_conductance')
    write(6, *) "Conductance:", res%gtop, res%gbot
  end if

  open(unit=10, file='site.txt')
  do i = 1, t
    write(10, 111) i, slabel(i), csize(i + 1)
  end do
  close(10)
  call perc_check(perc_ctx_destroy(h), 'perc_ctx_destroy')

111 format(i10, ",", i10, ",", i10)
121 format(i10, ",", i10)
end program site
