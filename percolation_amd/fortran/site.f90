! site.f90 -- drop-in for Fortran/Square/site.f and Fortran/Triangular/
! site.f: one site-percolation realisation filled to ps and its spanning
! test, on libperc.  With conductance = .true. (namelist) it also computes
! the ConductCalc.m site-rule conductance (MATLAB/ConductCalc.m:88-130),
! which the Fortran reference does not have.
!
! Parameters: the reference's block (Square/site.f:51-131: 50x50, ps = .60,
! seed 1080115; Triangular: ps = .548, seed 143285), overridable by an
! optional namelist file site.nml (&site_nml lattice, m, n, pbc, ps, seed,
! conductance, Va, g0, tol, itmax, device, trace /).  Outputs as the
! reference: bondlist.txt (i10,",",i10), siteorder.txt (list-directed),
! site.txt (j, s(j), c(j); site.f:353-358); trace = 1 also writes the
! per-site log siteocc.txt (site.f:167-350) from the host replay, before the
! device is opened.
program site
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
  integer(c_int) :: lattice, m, n, pbc, seed, itmax, device
  double precision :: ps, Va, g0, tol
  logical :: conductance
  integer(c_int) :: trace
  namelist /site_nml/ lattice, m, n, pbc, ps, seed, conductance, Va, g0, tol, itmax, device, trace
  integer(c_int) :: t, nb, tsites, i, rc, stats(4)
  integer(c_int), allocatable, target :: b1(:), b2(:), order(:), slabel(:), csize(:), rec(:)
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
  trace = 0
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
  if (trace /= 0) call write_siteocc()
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

contains

  ! siteocc.txt as the reference writes it (site.f:167-350): each site's
  ! step from perc_replay_site_trace, then the largest cluster and the
  ! spanning test over clusters of at least n sites in label order, from the
  ! host replay's numbering (perc_replay_labels)
  subroutine write_siteocc()
    integer(c_int) :: j, k, r, scn, sstats(4)
    integer(c_int), allocatable, target :: s(:), c(:)
    double precision :: f   ! site.f:40 (a double holding a single-precision quotient)
    scn = 4
    if (lattice /= PERC_SQUARE) scn = 6
    allocate(rec(PERC_SITE_TRACE * max(tsites, 1)), s(t), c(t + nb + 2))
    call perc_check(perc_replay_site_trace(lattice, m, n, pbc, tsites, c_loc(order), c_loc(rec)), &
                    'perc_replay_site_trace')
    call perc_check(perc_replay_labels(lattice, m, n, pbc, PERC_SITE, tsites, c_loc(order), 0, &
                                       c_null_ptr, c_null_ptr, c_loc(s), c_loc(c), t + nb + 2, &
                                       sstats), 'perc_replay_labels')
    open(unit=11, file='siteocc.txt')
    do i = 1, tsites
      r = PERC_SITE_TRACE * (i - 1)
      write(11, *) "site chosen:", rec(r + 1)
      write(11, *) "nearest neighbors:", (rec(r + 1 + j), j = 1, scn)
      write(11, *) "n.n. with largest cluster:", rec(r + 8)
      write(11, *) "largest cluster number:", rec(r + 9)
      write(11, *) "largest neighbor cluster size:", rec(r + 10)
      if (rec(r + 10) == 0) then
        write(11, *) "*no n.n. occupied*"
        write(11, *) "site assigned to cluster number", rec(r + 22)
      else
        write(11, *) "*one or more n.n. occupied*"
        do k = 1, rec(r + 11)
          write(11, *) "adding", rec(r + 10 + 2 * k), " to largest cluster"
          write(11, *) "largest cluster is now", rec(r + 11 + 2 * k)
        end do
        write(11, *) "site assigned to cluster number", rec(r + 22)
        write(11, *) "size of cluster number", rec(r + 22), " is now", rec(r + 23)
      end if
      f = real(i) / real(t)   ! site.f:267, single-precision division
      write(11, *) "fraction of lattice filled:", f
      write(11, *) "--------------------"
    end do
    call perc_log_spanning(11, sstats, c, s, m, t, n, .false.)
    close(11)
  end subroutine write_siteocc
end program site
