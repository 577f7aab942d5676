! bond_cond.f90 -- drop-in for Fortran/Square/bond_cond.f and Fortran/
! Triangular/bond_cond.f: for each trial ii (seed tseed(ii) from the master
! seed, bond_cond.f:62-70) the bond order is shuffled and the conductance
! of the lowest-label spanning cluster is computed at each grid point
! nbarr(jj) = pbarr(jj)*nb (square .49 + 5e-3 steps, 103 points;
! triangular .35, 131 points), then pc = first spanning fraction and the
! final spanning label are reported (bond_cond.f:123-498).
!
! The reference re-labels bond by bond and checks spanning after every
! bond; here each grid point is one GPU occupancy + labeling, pc is the
! smallest spanning occupation found by bisection (spanning is monotone in
! bf), and the conductance is the HIP Jacobi-PCG in linbcg order.  A grid
! value equal to the previous one stalls the sweep exactly as the
! reference's `bf == nbarr(jj)` test does (hazard H3).
!
! Parameters: the reference's block (10x10, numtrials 1, master seed 58302),
! overridable by bond_cond.nml (&bond_cond_nml lattice, m, n, pbc,
! numtrials, seed, Va, g0, tol, itmax, device, ndev, workers /).  Output: bondcond.txt as
! the reference writes it (bond_cond.f:107-117, 481-496).
!
! ndev >= 1 shards the trials over devices 0..ndev-1 of the node
! (perc_ensemble_bond_cond: trial ii on device (ii-1) mod ndev, one host
! thread each, rows gathered in ii order) and all-reduces the per-grid-point
! statistics with RCCL; bondcond.txt is the same file, and the reduced
! statistics go to bondcond_stats.txt.  ndev = 0 (default) runs every trial
! on `device` in this thread.  workers > 1 (with ndev >= 1) runs that many
! trials at a time on each device (perc_ensemble_set_workers: a context,
! host thread and stream each) -- small lattices leave a device mostly idle.
program bond_cond
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
  integer(c_int) :: lattice, m, n, pbc, numtrials, seed, itmax, device, ndev, workers
  double precision :: Va, g0, tol
  namelist /bond_cond_nml/ lattice, m, n, pbc, numtrials, seed, Va, g0, tol, itmax, device, &
                           ndev, workers
  integer(c_int) :: t, nb, i, ii, jj, bf, lastbf, npts, lo, hi, mid, bfc, perccln, stats(4)
  integer(c_int) :: tseed(1000), nbarr(250)
  double precision :: pbarr(250), pb, pc, Gtop, Gbot
  integer(c_int), allocatable, target :: order(:)
  type(c_ptr) :: h, ens
  integer(c_int), allocatable :: e_nrows(:), e_iters(:), e_bfc(:), e_pl(:)
  double precision, allocatable :: e_gbot(:), e_gtop(:), e_stats(:)
  double precision :: cnt, gm, gv
  type(perc_label_info) :: info
  type(perc_cond_result) :: res
  integer :: u

  lattice = PERC_LATTICE
  m = 10
  n = 10
  pbc = 0
  Va = 1.00d+00
  g0 = 1.00d+00
  numtrials = 1
  seed = 58302
  tol = 1.00d-08
  itmax = 2500
  device = 0
  ndev = 0
  workers = 1
  if (perc_have_file('bond_cond.nml')) then
    open(newunit=u, file='bond_cond.nml', status='old')
    read(u, nml=bond_cond_nml)
    close(u)
  end if
  if (numtrials < 1 .or. numtrials > 1000) error stop 'numtrials must be 1..1000'

  call perc_trial_seeds(seed, 1000, tseed)
  t = m * n
  nb = perc_nbonds(lattice, m, n, pbc)
  pbarr = 0.00d+00
  nbarr = 0
  if (lattice == PERC_SQUARE) then
    pbarr(1) = 0.49d+00
    npts = 103
  else
    pbarr(1) = 0.35d+00
    npts = 131
  end if
  do i = 2, npts
    pbarr(i) = pbarr(i - 1) + 5.00d-03
  end do
  do i = 1, 250
    nbarr(i) = pbarr(i) * nb
  end do

  open(unit=10, file='bondcond.txt')
  write(10, *) "m =", m
  write(10, *) "n =", n
  write(10, *) "t =", t
  write(10, *) "pbc =", pbc
  write(10, *) "total number of bonds in the lattice:", nb
  write(10, *) "Va =", Va
  write(10, *) "g0 =", g0
  write(10, *) "total number of iterations:", numtrials
  write(10, *) "random number for generating the trial seeds:", seed
  write(10, *) "------------------------------"

  if (ndev >= 1) then
    allocate(e_nrows(numtrials), e_bfc(numtrials), e_pl(numtrials))
    allocate(e_gbot(numtrials * 250), e_gtop(numtrials * 250), e_iters(numtrials * 250))
    allocate(e_stats(250 * 5))
    call perc_check(perc_ensemble_create(ndev, c_null_ptr, lattice, m, n, pbc, ens), &
                    'perc_ensemble_create')
    if (workers > 1) call perc_check(perc_ensemble_set_workers(ens, workers), &
                                     'perc_ensemble_set_workers')
    call perc_check(perc_ensemble_bond_cond(ens, numtrials, tseed, 250, nbarr, Va, g0, tol, &
                    itmax, e_nrows, e_gbot, e_gtop, e_iters, e_bfc, e_pl, e_stats), &
                    'perc_ensemble_bond_cond')
    call perc_check(perc_ensemble_destroy(ens), 'perc_ensemble_destroy')
    do ii = 1, numtrials   ! rows in trial order, as the serial loop writes them
      write(6, *) "Trial #", ii
      write(10, *) "Trial #", ii
      write(6, *) "Random number seed:", tseed(ii)
      write(10, *) "Random number seed:", tseed(ii)
      do jj = 1, e_nrows(ii)
        i = (ii - 1) * 250 + jj
        pb = real(nbarr(jj)) / real(nb)     ! REAL*4 quotient (bond_cond.f:351)
        write(6, 111) pb, e_gbot(i), e_gtop(i), ((e_gbot(i) + e_gtop(i)) / 2)
        write(10, 111) pb, e_gbot(i), e_gtop(i), ((e_gbot(i) + e_gtop(i)) / 2)
      end do
      pc = 0.00d+00
      if (e_bfc(ii) > 0) pc = real(e_bfc(ii)) / real(nb)
      write(6, *) "lattice-spanning cluster:", e_pl(ii)
      write(10, *) "lattice-spanning cluster:", e_pl(ii)
      write(6, *) "pc =", pc
      write(10, *) "pc =", pc
      write(6, *) "------------------------------"
      write(10, *) "------------------------------"
    end do
    close(10)
    ! ensemble statistics (RCCL all-reduced): pb, count, <Gtop>, var Gtop,
    ! spanning fraction, mean iterations
    open(unit=11, file='bondcond_stats.txt')
    write(11, '(a,i0)') 'devices: ', ndev
    do jj = 1, 250
      cnt = e_stats((jj - 1) * 5 + 1)
      if (cnt <= 0.0d0) exit
      gm = e_stats((jj - 1) * 5 + 2) / cnt
      gv = max(e_stats((jj - 1) * 5 + 3) / cnt - gm * gm, 0.0d0)
      pb = real(nbarr(jj)) / real(nb)
      write(11, 112) pb, int(cnt), gm, gv, e_stats((jj - 1) * 5 + 4) / cnt, &
                     e_stats((jj - 1) * 5 + 5) / cnt
    end do
    close(11)
    stop
  end if

  allocate(order(nb + 1))
  call perc_check(perc_ctx_create(device, lattice, m, n, pbc, h), 'perc_ctx_create')
  do ii = 1, numtrials
    write(6, *) "Trial #", ii
    write(10, *) "Trial #", ii
    write(6, *) "Random number seed:", tseed(ii)
    write(10, *) "Random number seed:", tseed(ii)
    call perc_shuffled_ids(nb, tseed(ii), order)

    jj = 1
    lastbf = -1
    do while (jj <= 250)
      bf = nbarr(jj)
      if (bf <= 0 .or. bf <= lastbf) exit
      call perc_check(perc_occupy(h, PERC_BOND, 0, c_null_ptr, bf, c_loc(order)), 'perc_occupy')
      call perc_check(perc_label(h, info, c_null_ptr), 'perc_label')
      call perc_check(perc_conductance(h, PERC_RULE_BOND, PERC_CUR_FORTRAN, Va, g0, PERC_LEAK, &
                                       2, tol, itmax, res, c_null_ptr), 'perc_conductance')
      Gtop = res%gtop
      Gbot = res%gbot
      pb = real(bf) / real(nb)               ! REAL*4 quotient (bond_cond.f:351)
      write(6, 111) pb, Gbot, Gtop, ((Gbot + Gtop) / 2)
      write(10, 111) pb, Gbot, Gtop, ((Gbot + Gtop) / 2)
      lastbf = bf
      jj = jj + 1
    end do

    ! pc: first occupation with a spanning cluster (bond_cond.f:381)
    call perc_check(perc_occupy(h, PERC_BOND, 0, c_null_ptr, nb, c_loc(order)), 'perc_occupy')
    call perc_check(perc_label(h, info, c_null_ptr), 'perc_label')
    bfc = 0
    perccln = 0
    if (info%nspan > 0) then
      ! final lowest spanning label (all bonds filled)
      call perc_check(perc_label_numbers(h, c_null_ptr, c_null_ptr, c_null_ptr, 0, stats), &
                      'perc_label_numbers')
      perccln = stats(4)
      lo = 0
      hi = nb
      do while (hi - lo > 1)
        mid = (lo + hi) / 2
        call perc_check(perc_occupy(h, PERC_BOND, 0, c_null_ptr, mid, c_loc(order)), &
                        'perc_occupy')
        call perc_check(perc_label(h, info, c_null_ptr), 'perc_label')
        if (info%nspan > 0) then
          hi = mid
        else
          lo = mid
        end if
      end do
      bfc = hi
    end if
    pc = 0.00d+00
    if (bfc > 0) pc = real(bfc) / real(nb)
    write(6, *) "lattice-spanning cluster:", perccln
    write(10, *) "lattice-spanning cluster:", perccln
    write(6, *) "pc =", pc
    write(10, *) "pc =", pc
    write(6, *) "------------------------------"
    write(10, *) "------------------------------"
  end do
  close(10)
  call perc_check(perc_ctx_destroy(h), 'perc_ctx_destroy')

111 format(f12.9, ",", f12.9, ",", f12.9, ",", f12.9)
112 format(f12.9, ",", i8, ",", es24.16, ",", es24.16, ",", f10.6, ",", f14.2)
end program bond_cond
