! perc_mixed_scan.f90 -- drop-in for Fortran/Square/sb_perc.f (-DPERC_SCAN_BS=0)
! and bs_perc.f (-DPERC_SCAN_BS=1), and their Triangular twins.
!
! For each point ii (sb: ps, bs: pb = start + step*(ii-1)) the trial seeds
! sseed(jj), bseed(jj) are drawn alternately after srand(pseed(ii))
! (sb_perc.f:94-111); for each of `iters` trials one kind is filled to the
! point's fraction and the other is added until a mixed cluster spans; the
! record is (sseed, bseed, ps, pb), the scanned fraction 0 if nothing spans
! (sb_perc.f:365-379, bs_perc.f:388-402).
!   sb_perc: first spanning bond count by perc_first_spanning_mixed (GPU
!            labeling in a bisection).
!   bs_perc: the reference as built reads c(0) out of bounds (hazard H11,
!            perc.h); its scan is reproduced by perc_bs_perc_replay
!            (as_built = .true., default) or, as_built = .false., the
!            intended site+bond connectivity on the GPU.
!
! Parameters: the reference's blocks (sb: 50x50, seed 8811064, ps 0.59 +
! 0.01 i x 42 (triangular 0.50 + 0.01 i x 51), iter 100; bs: 10x10, seed
! 229102, pb 0.30 + 0.01 i x 71, iter 1000), overridable by sb_perc.nml /
! bs_perc.nml (&mixed_scan_nml lattice, m, n, pbc, seed, pstart, pstep,
! npoints, iters, as_built, device /).
program perc_mixed_scan
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
#ifndef PERC_SCAN_BS
#define PERC_SCAN_BS 0
#endif
  integer(c_int) :: lattice, m, n, pbc, seed, npoints, iters, device
  double precision :: pstart, pstep
  logical :: as_built
  namelist /mixed_scan_nml/ lattice, m, n, pbc, seed, pstart, pstep, npoints, iters, as_built, &
                            device
  integer(c_int) :: t, nb, ii, jj, fixed, first, pseed(100), sseed(1000), bseed(1000)
  integer(c_int), allocatable, target :: sorder(:), border(:)
  double precision :: pt, ps, pb
  character(len=16) :: nml, out
  type(c_ptr) :: h
  integer :: u

  lattice = PERC_LATTICE
  pbc = 0
  as_built = .true.
  device = 0
  if (PERC_SCAN_BS == 1) then
    m = 10
    n = 10
    seed = 229102
    pstart = 0.30d+00
    pstep = 0.01d+00
    npoints = 71
    iters = 1000
    nml = 'bs_perc.nml'
    out = 'bs_perc.txt'
  else
    m = 50
    n = 50
    seed = 8811064
    if (lattice == PERC_SQUARE) then
      pstart = 0.59d+00
      npoints = 42
    else
      pstart = 0.50d+00
      npoints = 51
    end if
    pstep = 0.01d+00
    iters = 100
    nml = 'sb_perc.nml'
    out = 'sb_perc.txt'
  end if
  if (perc_have_file(trim(nml))) then
    open(newunit=u, file=trim(nml), status='old')
    read(u, nml=mixed_scan_nml)
    close(u)
  end if
  if (npoints < 1 .or. npoints > 100 .or. iters < 1 .or. iters > 1000) &
    error stop 'npoints must be 1..100 and iters 1..1000'

  t = m * n
  nb = perc_nbonds(lattice, m, n, pbc)
  allocate(sorder(t + 1), border(nb + 1))
  call perc_trial_seeds(seed, 100, pseed)
  call perc_check(perc_ctx_create(device, lattice, m, n, pbc, h), 'perc_ctx_create')
  open(unit=10, file=trim(out))
  do ii = 1, npoints
    pt = pstart + (pstep * (ii - 1))
    call perc_srand(pseed(ii))
    do jj = 1, 1000
      sseed(jj) = int(perc_rand(0) * 10000000) + 1
      bseed(jj) = int(perc_rand(0) * 10000000) + 1
    end do
    do jj = 1, iters
      call perc_shuffled_ids(t, sseed(jj), sorder)
      call perc_shuffled_ids(nb, bseed(jj), border)
      if (PERC_SCAN_BS == 1) then
        fixed = pt * nb
        if (as_built) then
          call perc_check(perc_bs_perc_replay(lattice, m, n, pbc, sorder, t, border, fixed, 1, &
                                              first), 'perc_bs_perc_replay')
        else
          call perc_check(perc_first_spanning_mixed(h, PERC_SITE, c_loc(sorder), t, &
                          c_loc(border), fixed, 0, first), 'perc_first_spanning_mixed')
        end if
        pb = real(fixed) / real(nb)
        ps = 0.00d+00
        if (first > 0) ps = real(first) / real(t)
      else
        fixed = pt * t
        call perc_check(perc_first_spanning_mixed(h, PERC_BOND, c_loc(sorder), fixed, &
                        c_loc(border), nb, 0, first), 'perc_first_spanning_mixed')
        ps = real(fixed) / real(t)
        pb = 0.00d+00
        if (first > 0) pb = real(first) / real(nb)
      end if
      write(6, 111) sseed(jj), bseed(jj), ps, pb
      write(10, 111) sseed(jj), bseed(jj), ps, pb
    end do
  end do
  close(10)
  call perc_check(perc_ctx_destroy(h), 'perc_ctx_destroy')
111 format(i10, ",", i10, ",", f12.9, ",", f12.9)
end program perc_mixed_scan
