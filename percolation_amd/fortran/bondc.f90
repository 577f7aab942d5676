! bondc.f90 -- drop-in for Fortran/Square/bondc.f and Fortran/Triangular/
! bondc.f: one bond-percolation realisation filled to pb, the spanning test
! and the conductance of the spanning cluster, on libperc.
!
! Parameters: the reference's block (Square/bondc.f:67-92; Triangular:
! pb = .35, seed = 62703), overridable by an optional namelist file
! bondc.nml (&bondc lattice, m, n, pbc, pb, seed, Va, g0, tol, itmax,
! device, nslab, xport, dot_order, condtype, cseed, trace /).  trace = 1 also
! writes the reference's per-bond log bondocc.txt (bondc.f:194-594; byte-
! identical with dot_order = 1, whose conductance line is the reference
! solver's bitwise).  condtype 2 gives the
! spanning cluster's bonds -g0*rand('twister', cseed) (MATLAB/ConductCalc.m
! condtype 2; 1, the default, fixed g0).  nslab > 1 splits the solve into row
! slabs over nslab contexts (devices device .. device+nslab-1 with xport 0,
! RCCL; all on `device` with xport 1, host-staged); the split solve runs the
! slab march, so it needs m a multiple of 128, fixed conductances (condtype
! 1: the stencil operator) and the fast dot order -- otherwise the driver
! warns on stderr and solves on one context (perc_conductance).  dot_order 1
! folds linbcg's sums in the reference's order (bitwise its solve).  Outputs as
! the reference: bondorder.txt (i10,",",i10) in
! shuffled order (bondc.f:177-180), bond.txt (b1, b2, label, j, c(j);
! bondc.f:600-604) and the run summary on stdout.
program bondc
  use perc_api
  implicit none
#ifndef PERC_LATTICE
#define PERC_LATTICE 0
#endif
  integer(c_int) :: lattice, m, n, pbc, seed, itmax, device, nslab, xport, dot_order, condtype, cseed
  integer(c_int) :: trace
  double precision :: pb, Va, g0, tol
  namelist /bondc_nml/ lattice, m, n, pbc, pb, seed, Va, g0, tol, itmax, device, nslab, xport, &
                       dot_order, condtype, cseed, trace
  integer(c_int), allocatable, target :: rec(:)
  integer :: botfill, topfill, k
  double precision :: fb    ! bondc.f:52 (a double holding a single-precision quotient)
  integer(c_int) :: nb, tbonds, i, j, id, rc, stats(4), perccln, perccls, s, dev
  integer(c_int), allocatable, target :: b1(:), b2(:), order(:), label(:), csize(:)
  type(c_ptr) :: h
  type(c_ptr), allocatable, target :: hs(:)
  type(perc_label_info) :: info
  type(perc_cond_result) :: res
  integer :: u

  ! reference parameter block
  lattice = PERC_LATTICE
  m = 50
  n = 50
  pbc = 0
  if (lattice == PERC_SQUARE) then
    pb = 0.50d+00
    seed = 626504
  else
    pb = 0.35d+00
    seed = 62703
  end if
  Va = 1.00d+00
  g0 = 1.00d+00
  tol = 1.00d-08            ! linbcg call, bondc.f:545
  itmax = 2500              ! linbcg call, bondc.f:545
  device = 0
  nslab = 1
  xport = PERC_XPORT_RCCL
  dot_order = PERC_DOT_FAST
  condtype = 1
  cseed = 1838534
  trace = 0
  if (perc_have_file('bondc.nml')) then
    open(newunit=u, file='bondc.nml', status='old')
    read(u, nml=bondc_nml)
    close(u)
  end if

  ! bond list in reference order and the shuffled bond order
  nb = perc_nbonds(lattice, m, n, pbc)
  allocate(b1(nb), b2(nb), order(nb + 1), label(nb), csize(nb + 2))
  rc = perc_bond_list(lattice, m, n, pbc, b1, b2)
  call perc_shuffled_ids(nb, seed, order)
  open(unit=12, file='bondorder.txt')
  do i = 1, nb
    id = order(i)
    if (id > 0) then
      write(12, 121) b1(id), b2(id)
    else
      write(12, 121) 0, 0
    end if
  end do
  close(12)

  ! occupy the first tbonds of the order, label on the GPU
  tbonds = pb * nb          ! bondc.f:191 (truncation)
  call perc_check(perc_ctx_create(device, lattice, m, n, pbc, h), 'perc_ctx_create')
  call perc_check(perc_occupy(h, PERC_BOND, 0, c_null_ptr, tbonds, c_loc(order)), 'perc_occupy')
  call perc_check(perc_label(h, info, c_null_ptr), 'perc_label')
  ! reference label numbers and cluster sizes (bond.txt) by host replay
  call perc_check(perc_label_numbers(h, c_loc(label), c_null_ptr, c_loc(csize), nb + 2, stats), &
                  'perc_label_numbers')
  perccln = stats(4)
  perccls = 0
  if (perccln > 0) perccls = csize(perccln + 1)
  if (trace /= 0) then
    ! bondocc.txt as the reference writes it (bondc.f:194-462): the per-bond
    ! steps from the host replay, then the spanning test over the clusters
    ! of at least n-1 bonds in label order
    allocate(rec(3 * max(tbonds, 1)))
    call perc_check(perc_replay_bond_trace(lattice, m, n, pbc, tbonds, c_loc(order), c_loc(rec)), &
                    'perc_replay_bond_trace')
    open(unit=11, file='bondocc.txt')
    do i = 1, tbonds
      id = order(i)
      if (id > 0) then
        write(11, *) "bond chosen:", b1(id), b2(id)
      else
        write(11, *) "bond chosen:", 0, 0
      end if
      if (rec(3 * i - 2) == 0) then
        write(11, *) "*no n.n. occupied*"
        write(11, *) "bond assigned to cluster number", rec(3 * i - 1)
      else
        write(11, *) "*one or more n.n. occupied*"
        write(11, *) "bond assigned to cluster number", rec(3 * i - 1)
        write(11, *) "size of cluster number", rec(3 * i - 1), " is now", rec(3 * i)
      end if
      fb = real(i) / real(nb)   ! bondc.f:371, single-precision division
      write(11, *) "fraction of lattice filled:", fb
      write(11, *) "--------------------"
    end do
    write(11, *)
    write(11, *) "******************************"
    write(11, *) "largest overall cluster number:", stats(2)
    write(11, *) "largest overall cluster size:", stats(3)
    s = 0
    do i = 1, stats(1) - 1
      if (csize(i + 1) >= n - 1) then
        write(11, *) "testing cluster:", i
        botfill = 0
        topfill = 0
        do k = 1, nb
          if (b1(k) <= m .and. label(k) == i) botfill = 1
          if (b2(k) > m * n - m .and. label(k) == i) topfill = 1
        end do
        if (botfill == 0) then
          write(11, *) "source end not connected"
          cycle
        end if
        if (topfill == 0) then
          write(11, *) "drain end not connected"
          cycle
        end if
        write(11, *) "infinite cluster present"
        write(11, *) "infinite cluster number:", i
        write(11, *) "infinite cluster size:", csize(i + 1)
        s = 1
        exit
      end if
    end do
    if (s == 0) write(11, *) "no infinite cluster present"
    write(11, *) "******************************"
  end if

  write(6, *)
  write(6, *) "******************************"
  write(6, *) "largest overall cluster number:", stats(2)
  write(6, *) "largest overall cluster size:", stats(3)
  if (perccln > 0) then
    write(6, *) "infinite cluster present"
    write(6, *) "infinite cluster number:", perccln
    write(6, *) "infinite cluster size:", perccls
  else
    write(6, *) "no infinite cluster present"
  end if
  write(6, *) "******************************"

  if (perccln > 0) then
    write(6, *) "Calculating internal node voltages"
    if (trace /= 0) write(11, *) "Calculating internal node voltages"
    if (dot_order /= PERC_DOT_FAST) call perc_check(perc_set_dot_order(h, dot_order), 'perc_set_dot_order')
    if (condtype == 2) call perc_check(perc_set_conductcalc_weights(h, PERC_RULE_BOND, cseed), &
                                       'perc_set_conductcalc_weights')
    if (nslab > 1 .and. (mod(m, 128) /= 0 .or. condtype == 2 .or. dot_order /= PERC_DOT_FAST)) then
      write(0, '(a)') 'bondc: nslab > 1 needs m a multiple of 128, condtype 1 and dot_order 0;' // &
                      ' solving on one context'
      nslab = 1
    end if
    if (nslab > 1) then
      ! the same occupancy labeled on every slab's context, then one split solve
      allocate(hs(nslab))
      hs(1) = h
      do s = 2, nslab
        dev = device
        if (xport == PERC_XPORT_RCCL) dev = device + s - 1
        call perc_check(perc_ctx_create(dev, lattice, m, n, pbc, hs(s)), 'perc_ctx_create')
        call perc_check(perc_occupy(hs(s), PERC_BOND, 0, c_null_ptr, tbonds, c_loc(order)), 'perc_occupy')
        call perc_check(perc_label(hs(s), info, c_null_ptr), 'perc_label')
        if (condtype == 2) call perc_check(perc_set_conductcalc_weights(hs(s), PERC_RULE_BOND, cseed), &
                                           'perc_set_conductcalc_weights')
      end do
      call perc_check(perc_dslab_solve_group(nslab, c_loc(hs), xport, PERC_RULE_BOND, PERC_CUR_FORTRAN, &
                                             Va, g0, PERC_LEAK, 2, tol, itmax, 0, res), &
                      'perc_dslab_solve_group')
      do s = 2, nslab
        call perc_check(perc_ctx_destroy(hs(s)), 'perc_ctx_destroy')
      end do
      deallocate(hs)
    else
      call perc_check(perc_conductance(h, PERC_RULE_BOND, PERC_CUR_FORTRAN, Va, g0, PERC_LEAK, &
                                       2, tol, itmax, res, c_null_ptr), 'perc_conductance')
    end if
    write(6, *) "Calculating currents"
    write(6, *) "--------------------"
    write(6, *) "Conductance:", res%gtop, res%gbot
    write(6, *) "linbcg iterations:", res%iter, " err:", res%err
    if (trace /= 0) then
      write(11, *) "Calculating currents"
      write(11, *) "--------------------"
      write(11, *) "Conductance:", res%gtop, res%gbot
    end if
  end if
  if (trace /= 0) close(11)

  open(unit=10, file='bond.txt')
  do j = 1, nb
    write(10, 111) b1(j), b2(j), label(j), j, csize(j + 1)
  end do
  close(10)
  call perc_check(perc_ctx_destroy(h), 'perc_ctx_destroy')

111 format(i10, ",", i10, ",", i10, ",", i10, ",", i10)
121 format(i10, ",", i10)
end program bondc
