! perc_mod.f90 -- ISO_C_BINDING interface of libperc (include/perc.h) for
! the Fortran drivers.  The drivers keep the reference programs' parameter
! blocks, RNG stream and output files (Fortran/Square/bondc.f,
! bond_cond.f, site.f, sitebond.f and their Triangular twins); the O(N^2)
! labeling loops, the dense Kirchhoff matrix, sprsin and linbcg are replaced
! by the libperc calls below (GPU labeling + host label replay + HIP
! Jacobi-PCG).
module perc_api
  use, intrinsic :: iso_c_binding
  implicit none

  integer(c_int), parameter :: PERC_OK = 0
  integer(c_int), parameter :: PERC_SQUARE = 0, PERC_TRIANGULAR = 1
  integer(c_int), parameter :: PERC_BOND = 0, PERC_SITE = 1, PERC_SITEBOND = 2, &
                                PERC_BONDSITE = 3
  ! ints per site of perc_replay_site_trace (siteocc.txt)
  integer(c_int), parameter :: PERC_SITE_TRACE = 24
  integer(c_int), parameter :: PERC_RULE_BOND = 0, PERC_RULE_SITE = 1, PERC_RULE_MIXED = 2
  integer(c_int), parameter :: PERC_CUR_FORTRAN = 0, PERC_CUR_MATLAB = 1
  ! association of linbcg's dot products (perc_set_dot_order)
  integer(c_int), parameter :: PERC_DOT_FAST = 0, PERC_DOT_LITERAL = 1, PERC_DOT_LITERAL_HOST = 2
  ! transports of the split solve (perc_dslab_solve_group)
  integer(c_int), parameter :: PERC_XPORT_RCCL = 0, PERC_XPORT_HOST = 1, PERC_XPORT_EXCHANGE = 4
  ! bytes of the RCCL unique id of the one-process-per-GPU split solve
  integer(c_int), parameter :: PERC_DSLAB_ID_BYTES = 128
  ! off-diagonal value of bonds outside the spanning cluster (bondc.f:487)
  real(c_double), parameter :: PERC_LEAK = 1.0d-12

  type, bind(C) :: perc_label_info
    integer(c_int) :: nclusters, nspan, span_root, span_sites, replayed, perccln
  end type perc_label_info

  type, bind(C) :: perc_cond_result
    real(c_double) :: gtop, gbot, err
    integer(c_int) :: iter, status
    real(c_double) :: t_assemble_ms, t_solve_ms, t_currents_ms
  end type perc_cond_result

  interface
    subroutine perc_srand(seed) bind(C, name='perc_srand')
      import :: c_int
      integer(c_int), value :: seed
    end subroutine perc_srand

    real(c_float) function perc_rand(i) bind(C, name='perc_rand')
      import :: c_int, c_float
      integer(c_int), value :: i
    end function perc_rand

    subroutine perc_trial_seeds(master, k, tseed) bind(C, name='perc_trial_seeds')
      import :: c_int
      integer(c_int), value :: master, k
      integer(c_int) :: tseed(*)
    end subroutine perc_trial_seeds

    subroutine perc_trial_seeds_scaled(master, k, scale, tseed) &
        bind(C, name='perc_trial_seeds_scaled')
      import :: c_int
      integer(c_int), value :: master, k, scale
      integer(c_int) :: tseed(*)
    end subroutine perc_trial_seeds_scaled

    integer(c_int) function perc_first_spanning(h, kind, order, nn, on_device, first) &
        bind(C, name='perc_first_spanning')
      import :: c_int, c_ptr
      type(c_ptr), value :: h, order
      integer(c_int), value :: kind, nn, on_device
      integer(c_int) :: first
    end function perc_first_spanning

    integer(c_int) function perc_first_spanning_mixed(h, scan, site_order, nsites, &
        bond_order, nbond, on_device, first) bind(C, name='perc_first_spanning_mixed')
      import :: c_int, c_ptr
      type(c_ptr), value :: h, site_order, bond_order
      integer(c_int), value :: scan, nsites, nbond, on_device
      integer(c_int) :: first
    end function perc_first_spanning_mixed

    integer(c_int) function perc_bs_perc_replay(lattice, m, n, pbc, site_order, nsites, &
        bond_order, nbond, c0_overflow, first) bind(C, name='perc_bs_perc_replay')
      import :: c_int
      integer(c_int), value :: lattice, m, n, pbc, nsites, nbond, c0_overflow
      integer(c_int) :: site_order(*), bond_order(*)
      integer(c_int) :: first
    end function perc_bs_perc_replay

    integer(c_int) function perc_replay_labels(lattice, m, n, pbc, kind, nsites, site_order, &
        nbond, bond_order, bond_label, site_label, csize, cap, stats) &
        bind(C, name='perc_replay_labels')
      import :: c_int, c_ptr
      integer(c_int), value :: lattice, m, n, pbc, kind, nsites, nbond, cap
      type(c_ptr), value :: site_order, bond_order, bond_label, site_label, csize
      integer(c_int) :: stats(4)
    end function perc_replay_labels

    ! bondc.f's per-bond trace records (bondocc.txt): 3 per order entry
    integer(c_int) function perc_replay_bond_trace(lattice, m, n, pbc, nbond, bond_order, trace) &
        bind(C, name='perc_replay_bond_trace')
      import :: c_int, c_ptr
      integer(c_int), value :: lattice, m, n, pbc, nbond
      type(c_ptr), value :: bond_order, trace
    end function perc_replay_bond_trace

    ! site.f's per-site steps (siteocc.txt): PERC_SITE_TRACE ints per site
    integer(c_int) function perc_replay_site_trace(lattice, m, n, pbc, nsite, site_order, trace) &
        bind(C, name='perc_replay_site_trace')
      import :: c_int, c_ptr
      integer(c_int), value :: lattice, m, n, pbc, nsite
      type(c_ptr), value :: site_order, trace
    end function perc_replay_site_trace

    ! sitebond.f / bondsite.f debug logs (sbdebug.txt / bsdebug.txt): event stream
    integer(c_int) function perc_replay_mixed_trace(lattice, m, n, pbc, kind, nsites, site_order, &
                                                    nbonds, bond_order, trace, cap, len) &
        bind(C, name='perc_replay_mixed_trace')
      import :: c_int, c_ptr, c_long_long
      integer(c_int), value :: lattice, m, n, pbc, kind, nsites, nbonds
      type(c_ptr), value :: site_order, bond_order, trace
      integer(c_long_long), value :: cap
      integer(c_long_long) :: len
    end function perc_replay_mixed_trace

    integer(c_int) function perc_nbonds(lattice, m, n, pbc) bind(C, name='perc_nbonds')
      import :: c_int
      integer(c_int), value :: lattice, m, n, pbc
    end function perc_nbonds

    integer(c_int) function perc_bond_list(lattice, m, n, pbc, b1, b2) &
        bind(C, name='perc_bond_list')
      import :: c_int
      integer(c_int), value :: lattice, m, n, pbc
      integer(c_int) :: b1(*), b2(*)
    end function perc_bond_list

    subroutine perc_shuffle(nn, order) bind(C, name='perc_shuffle')
      import :: c_int
      integer(c_int), value :: nn
      integer(c_int) :: order(*)
    end subroutine perc_shuffle

    integer(c_int) function perc_ctx_create(device, lattice, m, n, pbc, h) &
        bind(C, name='perc_ctx_create')
      import :: c_int, c_ptr
      integer(c_int), value :: device, lattice, m, n, pbc
      type(c_ptr) :: h
    end function perc_ctx_create

    integer(c_int) function perc_ctx_destroy(h) bind(C, name='perc_ctx_destroy')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function perc_ctx_destroy

    type(c_ptr) function perc_last_error() bind(C, name='perc_last_error')
      import :: c_ptr
    end function perc_last_error

    ! array arguments are pointers so that unused ones can be c_null_ptr
    integer(c_int) function perc_occupy(h, kind, nsites, site_order, nbond, bond_order) &
        bind(C, name='perc_occupy')
      import :: c_int, c_ptr
      type(c_ptr), value :: h, site_order, bond_order
      integer(c_int), value :: kind, nsites, nbond
    end function perc_occupy

    integer(c_int) function perc_label(h, info, canon_out) bind(C, name='perc_label')
      import :: c_int, c_ptr, perc_label_info
      type(c_ptr), value :: h, canon_out
      type(perc_label_info) :: info
    end function perc_label

    integer(c_int) function perc_label_numbers(h, bond_label, site_label, csize, cap, stats) &
        bind(C, name='perc_label_numbers')
      import :: c_int, c_ptr
      type(c_ptr), value :: h, bond_label, site_label, csize
      integer(c_int), value :: cap
      integer(c_int) :: stats(4)
    end function perc_label_numbers

    integer(c_int) function perc_cluster_sizes(h, maxcs, span_size) &
        bind(C, name='perc_cluster_sizes')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int) :: maxcs, span_size
    end function perc_cluster_sizes

    integer(c_int) function perc_conductance(h, rule, cur_rule, Va, g0, leak, itol, tol, &
        itmax, res, vint_out) bind(C, name='perc_conductance')
      import :: c_int, c_ptr, c_double, perc_cond_result
      type(c_ptr), value :: h, vint_out
      integer(c_int), value :: rule, cur_rule, itol, itmax
      real(c_double), value :: Va, g0, leak, tol
      type(perc_cond_result) :: res
    end function perc_conductance

    integer(c_int) function perc_set_dot_order(h, order) bind(C, name='perc_set_dot_order')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: order
    end function perc_set_dot_order

    ! what the last solve ran: out4 = (kernel PERC_RAN_*, flags, iterations, 0)
    integer(c_int) function perc_last_solve(h, out4) bind(C, name='perc_last_solve')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), intent(out) :: out4(4)
    end function perc_last_solve

    ! one solve split over K labeled contexts (row slabs, one host thread per
    ! context, RCCL or host-staged exchange): the linbcg call of bondc.f:545
    ! over several GPUs
    integer(c_int) function perc_dslab_solve_group(K, ctxs, xport, rule, cur_rule, Va, g0, leak, &
        itol, tol, itmax, full_x, res) bind(C, name='perc_dslab_solve_group')
      import :: c_int, c_ptr, c_double, perc_cond_result
      integer(c_int), value :: K, xport, rule, cur_rule, itol, itmax, full_x
      type(c_ptr), value :: ctxs
      real(c_double), value :: Va, g0, leak, tol
      type(perc_cond_result) :: res
    end function perc_dslab_solve_group

    ! ConductCalc.m condtype 2: the spanning cluster's bonds get -g0*rand('twister', seed)
    integer(c_int) function perc_set_conductcalc_weights(h, rule, seed) &
        bind(C, name='perc_set_conductcalc_weights')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
      integer(c_int), value :: rule, seed
    end function perc_set_conductcalc_weights

    ! the same loop with one process per GPU (an MPI program: rank 0 calls
    ! perc_dslab_unique_id, MPI_Bcast's the PERC_DSLAB_ID_BYTES bytes, every
    ! rank binds its labeled context to slab s of K, then perc_dslab_solve)
    integer(c_int) function perc_dslab_unique_id(id, nbytes) bind(C, name='perc_dslab_unique_id')
      import :: c_int, c_ptr
      type(c_ptr), value :: id
      integer(c_int), value :: nbytes
    end function perc_dslab_unique_id
    integer(c_int) function perc_dslab_comm_init(h, K, s, id, nbytes) bind(C, name='perc_dslab_comm_init')
      import :: c_int, c_ptr
      type(c_ptr), value :: h, id
      integer(c_int), value :: K, s, nbytes
    end function perc_dslab_comm_init
    integer(c_int) function perc_dslab_comm_free(h) bind(C, name='perc_dslab_comm_free')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function perc_dslab_comm_free
    integer(c_int) function perc_dslab_solve(h, rule, cur_rule, Va, g0, leak, itol, tol, itmax, &
        full_x, res) bind(C, name='perc_dslab_solve')
      import :: c_int, c_ptr, c_double, perc_cond_result
      type(c_ptr), value :: h
      integer(c_int), value :: rule, cur_rule, itol, itmax, full_x
      real(c_double), value :: Va, g0, leak, tol
      type(perc_cond_result) :: res
    end function perc_dslab_solve

    ! multi-GPU ensemble: one host thread + context per device, RCCL stats
    integer(c_int) function perc_ensemble_create(ndev, devices, lattice, m, n, pbc, e) &
        bind(C, name='perc_ensemble_create')
      import :: c_int, c_ptr
      integer(c_int), value :: ndev, lattice, m, n, pbc
      type(c_ptr), value :: devices
      type(c_ptr) :: e
    end function perc_ensemble_create

    integer(c_int) function perc_ensemble_destroy(e) bind(C, name='perc_ensemble_destroy')
      import :: c_int, c_ptr
      type(c_ptr), value :: e
    end function perc_ensemble_destroy

    integer(c_int) function perc_ensemble_set_workers(e, workers) &
        bind(C, name='perc_ensemble_set_workers')
      import :: c_int, c_ptr
      type(c_ptr), value :: e
      integer(c_int), value :: workers
    end function perc_ensemble_set_workers

    integer(c_int) function perc_ensemble_bond_cond(e, ntrials, tseed, npts, nbarr, Va, g0, &
        tol, itmax, nrows, gbot, gtop, iters, bf_c, perccln, stats) &
        bind(C, name='perc_ensemble_bond_cond')
      import :: c_int, c_ptr, c_double
      type(c_ptr), value :: e
      integer(c_int), value :: ntrials, npts, itmax
      real(c_double), value :: Va, g0, tol
      integer(c_int) :: tseed(*), nbarr(*), nrows(*), iters(*), bf_c(*), perccln(*)
      real(c_double) :: gbot(*), gtop(*), stats(*)
    end function perc_ensemble_bond_cond
  end interface

contains

  ! The reference `pause`s on errors; libperc returns a status instead.
  subroutine perc_check(rc, what)
    integer(c_int), intent(in) :: rc
    character(*), intent(in) :: what
    character(kind=c_char), pointer :: msg(:)
    integer :: k
    if (rc == PERC_OK) return
    call c_f_pointer(perc_last_error(), msg, [4096])
    k = 0
    do while (msg(k + 1) /= c_null_char .and. k < 4096)
      k = k + 1
    end do
    write(0, '(a,a,i0,a)') what, ' failed: status ', rc, ' ('
    write(0, *) msg(1:k), ')'
    error stop 1
  end subroutine perc_check

  ! 1-based id permutation of 1..nn after srand(seed): the reference's
  ! REAL*4 Fisher-Yates (bondc.f:162-174, site.f:131-147) with its spill
  ! slot nn+1 (hazard H2: a draw of j = nn+1 swaps in a 0 sentinel).
  subroutine perc_shuffled_ids(nn, seed, order)
    integer(c_int), intent(in) :: nn, seed
    integer(c_int), intent(out) :: order(nn + 1)
    integer(c_int) :: i
    do i = 1, nn
      order(i) = i
    end do
    order(nn + 1) = 0
    call perc_srand(seed)
    call perc_shuffle(nn, order)
  end subroutine perc_shuffled_ids

  ! the trace logs' closing block (site.f:295-350, sitebond.f:408-465,
  ! bondsite.f:358-418): largest cluster, then clusters 1..cln-1 of at least
  ! minsize elements in label order tested for a bottom- and a top-row site
  ! until one spans.  c(i + 1) is cluster i's size, s(1:t) the site labels;
  ! numbered: the mixed programs print "testing cluster", i
  subroutine perc_log_spanning(u, stats, c, s, m, t, minsize, numbered)
    integer, intent(in) :: u
    integer(c_int), intent(in) :: stats(4), c(:), s(:), m, t, minsize
    logical, intent(in) :: numbered
    integer(c_int) :: i
    logical :: span
    write(u, *)
    write(u, *) "******************************"
    write(u, *) "largest overall cluster number:", stats(2)
    write(u, *) "largest overall cluster size:", stats(3)
    span = .false.
    do i = 1, stats(1) - 1
      if (c(i + 1) < minsize) cycle
      if (numbered) then
        write(u, *) "testing cluster", i
      else
        write(u, *) "testing cluster"
      end if
      if (.not. any(s(1:m) == i)) then
        write(u, *) "source end not connected"
        cycle
      end if
      if (.not. any(s(t - m + 1:t) == i)) then
        write(u, *) "drain end not connected"
        cycle
      end if
      write(u, *) "infinite cluster present"
      write(u, *) "infinite cluster number:", i
      write(u, *) "infinite cluster size:", c(i + 1)
      span = .true.
      exit
    end do
    if (.not. span) write(u, *) "no infinite cluster present"
    write(u, *) "******************************"
  end subroutine perc_log_spanning

  ! an optional NAMELIST file overrides the reference parameter block
  logical function perc_have_file(name)
    character(*), intent(in) :: name
    inquire(file=name, exist=perc_have_file)
  end function perc_have_file
end module perc_api
