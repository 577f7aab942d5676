! sitebond.f90 -- drop-in for Fortran/Square/sitebond.f and Fortran/
! Triangular/sitebond.f: sites filled to ps (seed sseed), then bonds to pb
! (seed bseed), mixed labeling and spanning test, on libperc.  With
! conductance = .true. it also computes the ConductCalc.m mixed-rule
! conductance (MATLAB/ConductCalc.m:132-165).
!
! Parameters: the reference's block (Square/sitebond.f:54-71: 50x50,
! Triangular 10x10; ps = pb = .50, sseed 143285, bseed 43716), overridable
! by an optional namelist file sitebond.nml (&sitebond_nml lattice, m, n,
! pbc, ps, pb, sseed, bseed, conductance, Va, g0, tol, itmax, device,
! trace /).  Outputs as the reference: sbsite.txt (i, s(i), c(i)) and
! sbbond.txt (b1, b2, label) (sitebond.f:468-477); trace = 1 also writes the
! debug log sbdebug.txt (sitebond.f:184-465) from the host replay, before
! the device is opened.
program sitebond
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
  integer(c_int) :: lattice, m, n, pbc, sseed, bseed, itmax, device
  double precision :: ps, pb, Va, g0, tol
  logical :: conductance
  integer(c_int) :: trace
  namelist /sitebond_nml/ lattice, m, n, pbc, ps, pb, sseed, bseed, conductance, Va, g0, tol, &
                          itmax, device, trace
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
  trace = 0
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
  if (trace /= 0) call write_sbdebug()

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

contains

  ! sbdebug.txt as the reference writes it (sitebond.f:184-465): the site
  ! phase, each bond's step from perc_replay_mixed_trace's event stream (the
  ! record layout is in include/perc.h), then the closing block from the
  ! host replay's numbering
  subroutine write_sbdebug()
    integer(c_int), allocatable, target :: ev(:), s(:), c(:), bl(:)
    integer(c_int) :: r, k, e, id, sstats(4)
    integer(c_long_long) :: len
    double precision :: f   ! sitebond.f:44 (a double holding a single-precision quotient)
    call perc_check(perc_replay_mixed_trace(lattice, m, n, pbc, PERC_SITEBOND, ts, c_loc(sorder), &
                                            tb, c_loc(border), c_null_ptr, 0_c_long_long, len), &
                    'perc_replay_mixed_trace')
    allocate(ev(max(len, 1_c_long_long)), s(t), c(t + nb + 2), bl(nb))
    call perc_check(perc_replay_mixed_trace(lattice, m, n, pbc, PERC_SITEBOND, ts, c_loc(sorder), &
                                            tb, c_loc(border), c_loc(ev), len, len), &
                    'perc_replay_mixed_trace')
    call perc_check(perc_replay_labels(lattice, m, n, pbc, PERC_SITEBOND, ts, c_loc(sorder), tb, &
                                       c_loc(border), c_loc(bl), c_loc(s), c_loc(c), t + nb + 2, &
                                       sstats), 'perc_replay_labels')
    open(unit=12, file='sbdebug.txt')
    write(12, *) "Specified fraction of sites to fill:", ps
    do i = 1, ts
      write(12, *) "Site occupied:", sorder(i)
    end do
    f = real(ts) / real(t)
    write(12, *) "Actual fraction of sites filled:", f
    write(12, *) "--------------------"
    write(12, *) "Specified fraction of bonds to fill:", pb
    r = 1
    do i = 1, tb
      id = border(i)
      if (id > 0) then
        write(12, *) "Bond occupied:", b1(id), b2(id)
      else
        write(12, *) "Bond occupied:", 0, 0
      end if
      e = ev(r)
      select case (e)
      case (0)
        write(12, *) "Sites at end of bond unoccupied"
        write(12, *) "Bond belongs to cluster", ev(r + 1)
        r = r + 2
      case (1, 2)
        write(12, *) "Only site", ev(r + 1), " is occupied"
        write(12, *) "Bond added to cluster", ev(r + 2)
        write(12, *) "Cluster", ev(r + 2), " is now size", ev(r + 3)
        r = r + 4
      case (3, 4, 5)
        write(12, *) "Both sites occupied"
        write(12, *) "Site", ev(r + 1), " belongs to cluster", ev(r + 2), " of size", ev(r + 3)
        write(12, *) "Site", ev(r + 4), " belongs to cluster", ev(r + 5), " of size", ev(r + 6)
        if (e == 3) then
          write(12, *) "Sites belong to same cluster"
          write(12, *) "Cluster", ev(r + 2), " is now size", ev(r + 7)
          r = r + 8
        else
          if (e == 4) then
            write(12, *) "Site", ev(r + 1), " belongs to a larger cluster"
          else
            write(12, *) "Site", ev(r + 4), " belongs to a larger or equal-sized cluster"
          end if
          r = r + 7
          ! (lcn, size, oldcn) follow the two member lists
          k = r + 1 + ev(r)
          k = k + 1 + ev(k)
          do id = 1, ev(r)
            write(12, *) "Site", ev(r + id), " is now in cluster", ev(k)
          end do
          r = r + 1 + ev(r)
          do id = 1, ev(r)
            write(12, *) "Bond", b1(ev(r + id)), b2(ev(r + id)), " is now in cluster", ev(k)
          end do
          write(12, *) "Bond added to cluster", ev(k)
          write(12, *) "Cluster", ev(k), " is now size", ev(k + 1)
          write(12, *) "Cluster", ev(k + 2), " is now size", 0
          r = k + 3
        end if
      case default  ! 6: the spill slot
        r = r + 1
      end select
      write(12, *) "--------------------"
    end do
    f = real(tb) / real(nb)
    write(12, *) "Actual fraction of bonds filled:", f
    call perc_log_spanning(12, sstats, c, s, m, t, 2 * n - 1, .true.)
    close(12)
  end subroutine write_sbdebug
end program sitebond
