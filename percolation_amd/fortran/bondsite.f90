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
! bondsite.nml (&bondsite_nml lattice, m, n, pbc, ps, pb, sseed, bseed /).
! Outputs as the reference: bssite.txt (i, s(i), c(i) for i = 1..nb) and
! bsbond.txt (b1, b2, label) (bondsite.f:420-430).  bsdebug.txt is not
! written.
program bondsite
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
  integer(c_int) :: lattice, m, n, pbc, sseed, bseed
  double precision :: ps, pb
  namelist /bondsite_nml/ lattice, m, n, pbc, ps, pb, sseed, bseed
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
end program bondsite
