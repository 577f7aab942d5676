! perc_scan.f90 -- drop-in for Fortran/Square/bond_perc.f and site_perc.f
! (and their Triangular twins), compiled as bond_perc_{sq,tri} with
! -DPERC_SCAN_SITE=0 and site_perc_{sq,tri} with -DPERC_SCAN_SITE=1.
!
! For each trial ii the order is shuffled from tseed(ii) = int(rand(0)*1e6)+1
! (bond_perc.f:68-74) and filled until a cluster spans; the reference then
! writes tseed, the fraction filled (REAL*4), the largest cluster size and
! the spanning cluster size (bond_perc.f:364-367, site_perc.f:258-260).
! The reference re-labels after every element and scans for spanning; here
! the first spanning count comes from perc_first_spanning (GPU labeling in a
! bisection, spanning being monotone in the count) and the cluster sizes at
! that count from perc_cluster_sizes (GPU; equal to the reference's c(label)
! of the largest and of the spanning cluster, tests/test_threshold_scan.py).
!
! Parameters: the reference's block (50x50, numtrials 10 for bond_perc /
! 1000 for site_perc, master seed 58302), overridable by bond_perc.nml /
! site_perc.nml (&perc_scan_nml lattice, m, n, pbc, numtrials, seed, device /).
program perc_scan
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
#ifndef PERC_SCAN_SITE
#define PERC_SCAN_SITE 0
#endif
  integer(c_int) :: lattice, m, n, pbc, numtrials, seed, device
  namelist /perc_scan_nml/ lattice, m, n, pbc, numtrials, seed, device
  integer(c_int) :: kind, nn, ii, first, cnt, perccls, maxcs, spansz
  integer(c_int), allocatable, target :: tseed(:), order(:)
  character(len=16) :: nml, out
  real :: f
  type(c_ptr) :: h
  integer :: u

  lattice = PERC_LATTICE
  m = 50
  n = 50
  pbc = 0
  seed = 58302
  device = 0
  if (PERC_SCAN_SITE == 1) then
    kind = PERC_SITE
    numtrials = 1000
    nml = 'site_perc.nml'
    out = 'site_perc.txt'
  else
    kind = PERC_BOND
    numtrials = 10
    nml = 'bond_perc.nml'
    out = 'bond_perc.txt'
  end if
  if (perc_have_file(trim(nml))) then
    open(newunit=u, file=trim(nml), status='old')
    read(u, nml=perc_scan_nml)
    close(u)
  end if
  if (numtrials < 1 .or. numtrials > 50000) error stop 'numtrials must be 1..50000'

  if (kind == PERC_BOND) then
    nn = perc_nbonds(lattice, m, n, pbc)
  else
    nn = m * n
  end if
  allocate(tseed(numtrials), order(nn + 1))
  call perc_trial_seeds_scaled(seed, numtrials, 1000000, tseed)
  call perc_check(perc_ctx_create(device, lattice, m, n, pbc, h), 'perc_ctx_create')
  open(unit=10, file=trim(out))
  do ii = 1, numtrials
    call perc_shuffled_ids(nn, tseed(ii), order)
    call perc_check(perc_first_spanning(h, kind, c_loc(order), nn, 0, first), &
                    'perc_first_spanning')
    cnt = first
    if (first == 0) cnt = nn
    ! cluster sizes at that step (the context is left occupied at cnt and
    ! labeled): largest cluster and spanning cluster, on the GPU
    call perc_check(perc_cluster_sizes(h, maxcs, spansz), 'perc_cluster_sizes')
    perccls = 0
    if (first > 0) perccls = spansz
    f = real(cnt) / real(nn)
    write(6, *) tseed(ii), f, maxcs, perccls
    write(10, 111) tseed(ii), f, maxcs, perccls
  end do
  close(10)
  call perc_check(perc_ctx_destroy(h), 'perc_ctx_destroy')
111 format(i10, ",", f12.9, ",", i10, ",", i10)
end program perc_scan
