! bondsite.f90 -- drop-in for Fortran/Square/bondsite.f and Fortran/
! Triangular/bondsite.f: bonds filled to pb (seed bseed), each a cluster of
! size 1, then sites to ps (seed sseed), each joining the clusters of its
! occupied neighbour bonds (Square/bondsite.f:170-322), and the spanning
! test (bondsite.f:364-415), on libperc's O(N alpha) replay
! (perc_replay_labels, PERC_BONDSITE).  The reference computes no
! conductance here, so neither does this program (no device needed).
!
! Parameters: the reference's block (bondsite.f:52-74: 10x10, ps = pb = .50,
! sseed 143285, bseed 43716, pbc 0), overridable by an optional namelist file
! bondsite.nml (&bondsite_nml lattice, m, n, pbc, ps, pb, sseed, bseed,
! trace /).  Outputs as the reference: bssite.txt (i, s(i), c(i) for
! i = 1..nb) and bsbond.txt (b1, b2, label) (bondsite.f:420-430); trace = 1
! also writes the debug log bsdebug.txt (bondsite.f:178-418).
program bondsite
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
  integer(c_int) :: lattice, m, n, pbc, sseed, bseed
  double precision :: ps, pb
  integer(c_int) :: trace
  namelist /bondsite_nml/ lattice, m, n, pbc, ps, pb, sseed, bseed, trace
  integer(c_int) :: t, nb, ts, tb, i, rc, stats(4), cap
  integer(c_int), allocatable, target :: b1(:), b2(:), sorder(:), border(:), slabel(:), &
                                         blabel(:), csize(:)
  integer :: u

  lattice = PERC_LATTICE
  m = 10
  n = 10
  pbc = 0
  ps = 0.50d+00
  pb = 0.50d+00
  sseed = 143285
  bseed = 43716
  trace = 0
  if (perc_have_file('bondsite.nml')) then
    open(newunit=u, file='bondsite.nml', status='old')
    read(u, nml=bondsite_nml)
    close(u)
  end if

  t = m * n
  nb = perc_nbonds(lattice, m, n, pbc)
  cap = t + nb + 2
  allocate(b1(nb), b2(nb), sorder(t + 1), border(nb + 1), slabel(t), blabel(nb), csize(cap))
  rc = perc_bond_list(lattice, m, n, pbc, b1, b2)
  call perc_shuffled_ids(t, sseed, sorder)    ! bondsite.f:116-127
  call perc_shuffled_ids(nb, bseed, border)   ! bondsite.f:153-166
  tb = pb * nb                                ! bondsite.f:179
  ts = ps * t                                 ! bondsite.f:215
  call perc_check(perc_replay_labels(lattice, m, n, pbc, PERC_BONDSITE, ts, c_loc(sorder), &
                                     tb, c_loc(border), c_loc(blabel), c_loc(slabel), &
                                     c_loc(csize), cap, stats), 'perc_replay_labels')
  if (trace /= 0) call write_bsdebug()

  write(6, *) "largest overall cluster number:", stats(2)
  write(6, *) "largest overall cluster size:", stats(3)
  if (stats(4) > 0) then
    write(6, *) "infinite cluster number:", stats(4)
    write(6, *) "infinite cluster size:", csize(stats(4) + 1)
  else
    write(6, *) "no infinite cluster present"
  end if

  open(unit=10, file='bssite.txt')
  do i = 1, nb
    if (i <= t) then
      write(10, 111) i, slabel(i), csize(i + 1)
    else
      write(10, 111) i, 0, csize(i + 1)
    end if
  end do
  close(10)
  open(unit=11, file='bsbond.txt')
  do i = 1, nb
    write(11, 111) b1(i), b2(i), blabel(i)
  end do
  close(11)

111 format(i10, ",", i10, ",", i10)

contains

  ! bsdebug.txt as the reference writes it (bondsite.f:178-418): the bond
  ! phase, each site's step from perc_replay_mixed_trace's event stream (the
  ! record layout is in include/perc.h), then the closing block
  subroutine write_bsdebug()
    integer(c_int), allocatable, target :: ev(:)
    integer(c_int) :: r, k, id
    integer(c_long_long) :: len
    double precision :: f   ! bondsite.f:44 (a double holding a single-precision quotient)
    call perc_check(perc_replay_mixed_trace(lattice, m, n, pbc, PERC_BONDSITE, ts, c_loc(sorder), &
                                            tb, c_loc(border), c_null_ptr, 0_c_long_long, len), &
                    'perc_replay_mixed_trace')
    allocate(ev(max(len, 1_c_long_long)))
    call perc_check(perc_replay_mixed_trace(lattice, m, n, pbc, PERC_BONDSITE, ts, c_loc(sorder), &
                                            tb, c_loc(border), c_loc(ev), len, len), &
                    'perc_replay_mixed_trace')
    open(unit=12, file='bsdebug.txt')
    write(12, *) "Specified fraction of bonds to fill:", pb
    do i = 1, tb
      id = border(i)
      if (id > 0) then
        write(12, *) "Bond occupied:", b1(id), b2(id)
      else
        write(12, *) "Bond occupied:", 0, 0
      end if
    end do
    f = real(tb) / real(nb)
    write(12, *) "Actual fraction of bonds filled:", f
    write(12, *) "===================="
    write(12, *) "Specified fraction of sites to fill:", ps
    r = 1
    do i = 1, ts
      write(12, *) "Site occupied:", sorder(i)
      if (ev(r) == 0) then
        write(12, *) "*no neighboring bonds are occupied*"
        write(12, *) "site assigned to cluster number", ev(r + 1)
        r = r + 2
      else
        write(12, *) "*one or more n.n. bonds occupied*"
        do k = 1, ev(r + 1)
          write(12, *) "adding", ev(r + 2 * k), " to largest cluster"
          write(12, *) "largest cluster is now", ev(r + 2 * k + 1)
        end do
        r = r + 2 + 2 * ev(r + 1)
        write(12, *) "site assigned to cluster number", ev(r)
        write(12, *) "size of cluster number", ev(r), " is now", ev(r + 1)
        r = r + 2
      end if
      write(12, *) "--------------------"
    end do
    f = real(ts) / real(t)
    write(12, *) "Actual fraction of sites filled:", f
    call perc_log_spanning(12, stats, csize, slabel, m, t, 2 * n - 1, .true.)
    close(12)
  end subroutine write_bsdebug
end program bondsite
