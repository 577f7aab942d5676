/*
 * perc.h -- libperc C-ABI: MI355X-native cluster labeling + Kirchhoff
 * conductance for the IsaiahSteinke/Percolation Fortran drivers.
 *
 * Plain C types only (int32 indices, fp64 values, caller-owned host arrays).
 * Every entry returns an int status (PERC_OK == 0) where the reference would
 * `pause` (Fortran/Square/bondc.f:737,777,891,906).  One context per device
 * and host thread; no hidden globals except the gfortran-compatible RNG
 * stream (perc_srand/perc_rand), which is process-global exactly like
 * libgfortran's rand/srand.
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   nearestn          Fortran/Square/bondc.f:617-715, Triangular/bondc.f:619-804
 *   bond list         Fortran/Square/bondc.f:137-154
 *   rand / srand      GNU Fortran runtime; call sites Square/bondc.f:162,167
 *   labeling loops    Square/bondc.f:194-393, Square/site.f:167-289,
 *                     Square/sitebond.f:187-400
 *   spanning test     Square/bondc.f:413-456, Square/site.f:309-344,
 *                     Square/sitebond.f:423-458
 *   assembly + solve  Square/bondc.f:465-595 (bond); MATLAB/ConductCalc.m:
 *                     88-196 (site / mixed weight rules)
 *   NR sparse layer   sprsin/linbcg/atimes/asolve/snrm/dsprsax/dsprstx,
 *                     Square/bondc.f:723-917 (symbols below, F77 ABI)
 */
#ifndef PERC_H
#define PERC_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define PERC_OK 0
#define PERC_EINVAL (-1)     /* bad argument                                  */
#define PERC_ENOMEM (-2)     /* device or host allocation failed              */
#define PERC_EHIP (-3)       /* HIP runtime error                             */
#define PERC_ENMAX (-4)      /* 'nmax too small in sprsin'  (bondc.f:737)     */
#define PERC_EITOL (-5)      /* 'illegal itol in linbcg'    (bondc.f:777)     */
#define PERC_EMISMATCH (-6)  /* 'mismatched vector and matrix' (bondc.f:891)  */
#define PERC_EREPLAY (-7)    /* label replay impossible (H7: odd-m triangular) */
#define PERC_ENODEV (-8)     /* no HIP device                                  */
#define PERC_ESTATE (-9)     /* call order violated (e.g. solve before label)  */

/* lattice kinds */
#define PERC_SQUARE 0
#define PERC_TRIANGULAR 1
/* occupancy kinds */
#define PERC_BOND 0
#define PERC_SITE 1
#define PERC_SITEBOND 2
#define PERC_BONDSITE 3  /* bonds first, then sites (Square/bondsite.f); perc_replay_labels only */
/* conductance weight rules (which bonds get g0; all others get `leak`) */
#define PERC_RULE_BOND 0     /* bond label == perccln         (bondc.f:483) */
#define PERC_RULE_SITE 1     /* both end sites in perccln     (ConductCalc.m:90) */
#define PERC_RULE_MIXED 2    /* bond and both sites in perccln (ConductCalc.m:136) */
/* terminal-current rules */
#define PERC_CUR_FORTRAN 0   /* sprsin(G,1e-10) + dsprsax, ascending sums (bondc.f:576-592) */
#define PERC_CUR_MATLAB 1    /* full G*V, Itop summed from site t down (ConductCalc.m:188-196) */

typedef struct perc_ctx perc_ctx;

/* ---- RNG: GNU Fortran rand/srand (Park-Miller 16807, 2^31-1) ----------- */
void perc_srand(int seed);
float perc_rand(int i);
/* tseed(1..k) = int(rand(0)*1e7)+1 after srand(master) (bond_cond.f:65-70) */
void perc_trial_seeds(int master, int k, int *tseed);
/* same with int(rand(0)*scale)+1: the threshold scans use scale 1e6
   (Square/bond_perc.f:70-74, Square/site_perc.f:71-75) */
void perc_trial_seeds_scaled(int master, int k, int scale, int *tseed);

/* ---- host-side lattice helpers --------------------------------------- */
int perc_nbonds(int lattice, int m, int n, int pbc);
/* nn[0..5] of site rn (1-based), 0 = none; returns scn */
int perc_nearestn(int lattice, int m, int n, int pbc, int rn, int *nn);
/* bond list b1[k] < b2[k], k = 0..nb-1 in reference order; returns nb */
int perc_bond_list(int lattice, int m, int n, int pbc, int *b1, int *b2);
/* REAL*4 Fisher-Yates of a 1-based id permutation, H2-exact: order has N+1
   slots; on entry order[k] = k+1 (k<N) and order[N] = 0; uses the global
   RNG stream from the current seed (Square/bondc.f:166-174). */
void perc_shuffle(int N, int *order);

/* ---- context --------------------------------------------------------- */
int perc_ctx_create(int device, int lattice, int m, int n, int pbc, perc_ctx **out);
int perc_ctx_destroy(perc_ctx *h);
/* last HIP error string for diagnostics (never NULL) */
const char *perc_last_error(void);
/* One HIP runtime per process: the number of distinct libamdhip64 objects
   mapped in the process (dl_iterate_phdr), their paths ';'-separated into
   buf (cap bytes, may be NULL), the copy libperc's own calls bind to
   (dladdr of hipGetDeviceCount) first.  Two copies -- e.g. /opt/rocm's,
   loaded with libperc, and a framework's bundled one loaded later -- share
   one device through two runtimes and corrupt the heap at process exit;
   perc_ctx_create refuses to run then (PERC_ESTATE, the paths in
   perc_last_error). */
int perc_hip_runtimes(char *buf, int cap);

/* ---- occupancy + labeling -------------------------------------------- */
/* Occupy the first `count` entries of `order` (1-based bond ids for
   PERC_BOND, site ids for PERC_SITE; 0 = H2 sentinel, skipped).  For
   PERC_SITEBOND both lists are given.  Host arrays, copied to the device. */
int perc_occupy(perc_ctx *h, int kind, int nsites, const int *site_order,
                int nbonds, const int *bond_order);

/* Same, with the order lists already resident in device memory (device
   pointers on the context's device); used when inputs live in HBM. */
int perc_occupy_device(perc_ctx *h, int kind, int nsites, const int *d_site_order,
                       int nbonds, const int *d_bond_order);

typedef struct {
  int nclusters;      /* connected components with >= 1 occupied element     */
  int nspan;          /* spanning components                                  */
  int span_root;      /* canonical id (min site) of the chosen spanning one, 0 */
  int span_sites;     /* sites in the chosen spanning component               */
  int replayed;       /* 1 if the host label replay decided the lowest label  */
  int perccln;        /* reference label of the chosen component if known     */
} perc_label_info;

/* Occupation drawn on the device, with no order array (the metric
   ensemble's inputs without a host draw or an upload): element id (1-based)
   gets the key (hash32(seed, id) << 32) | id and the nsites / nbonds
   smallest keys are occupied (a radix select, 8 passes of one key byte) --
   the first nsites / nbonds of the permutation "ids in ascending key
   order", a uniform random permutation up to the order of equal 32-bit
   hashes.  Bonds use the key stream of mix64(seed ^ 0x5DEECE66D).  A host
   replay (perc_label_numbers, several spanning clusters) regenerates the
   order on the host; perc_random_order gives it to a caller. */
int perc_occupy_random(perc_ctx *h, int kind, int nsites, int nbonds, unsigned long long seed);
int perc_random_order(long long n, int count, unsigned long long seed, int kind, int *order_out);

/* The occupancy in device memory, copied out (either output may be NULL):
   site_occ[t] (site ids 1..t), bond_occ[nb] (bond ids 1..nb), 0 / 1 each. */
int perc_occupancy(perc_ctx *h, unsigned char *site_occ, unsigned char *bond_occ);

/* GPU connected components of the occupancy + spanning detection.  When
   more than one component spans, the reference's lowest-label rule is
   resolved by the host replay (hazard H4).  canon_out (optional, host,
   t ints) receives the canonical component id (min site id, 0 = empty site)
   per site. */
int perc_label(perc_ctx *h, perc_label_info *info, int *canon_out);

/* Reference label numbers (history-dependent, Square/bondc.f:275-364) by
   O(N alpha) host replay of the last occupancy.  Any output may be NULL.
   bond_label[nb], site_label[t], csize[cap] (cap >= nb+2 bond, t+2 site,
   t+nb+2 mixed), stats[4] = {cln, maxcn, maxcs, perccln}. */
int perc_label_numbers(perc_ctx *h, int *bond_label, int *site_label,
                       int *csize, int cap, int *stats);

/* Cluster sizes of the labeled occupancy on the GPU (bond or site kind):
   *maxcs = the largest cluster's size and *span_size = the size of the
   spanning cluster perc_label chose (0 if none), in bonds for PERC_BOND
   (c(label) of Square/bond_perc.f:296-322) and sites for PERC_SITE
   (site_perc.f).  These are the maxcs / perccls columns of bond_perc.txt /
   site_perc.txt: the same numbers as perc_label_numbers' stats[2] and
   csize[perccln] (clusters only grow, so the running maximum is the final
   largest size), without the host replay. */
int perc_cluster_sizes(perc_ctx *h, int *maxcs, int *span_size);

/* Percolation threshold of one order (Square/bond_perc.f:204-366,
   Square/site_perc.f:150-256, Square/bond_cond.f:381 pc): *first = the
   smallest count c such that occupying order[0..c) (bond ids for PERC_BOND,
   site ids for PERC_SITE) has a spanning cluster, 0 if even all n do not.
   Bisection over c with the GPU labeling (spanning is monotone in c); the
   order is uploaded once (or is a device array when on_device != 0).  The
   context is left occupied at c (or n) and labeled, so perc_label_numbers
   gives the reference's maxcs / spanning-cluster size at that step. */
int perc_first_spanning(perc_ctx *h, int kind, const int *order, int n, int on_device,
                        int *first);

/* Mixed threshold scans (Square/sb_perc.f:104-372, Square/bs_perc.f:104-
   395): one kind fixed, the other scanned.  scan = PERC_BOND: sites
   site_order[0..nsites) occupied, *first = smallest c <= nbonds such that
   bonds bond_order[0..c) make a spanning mixed cluster (bonds connect sites
   whose ends are both occupied; spanning on bottom/top-row sites);
   scan = PERC_SITE: bonds bond_order[0..nbonds) fixed, sites scanned.  0 if
   nothing spans.  GPU labeling in a bisection; the context is left
   unoccupied. */
int perc_first_spanning_mixed(perc_ctx *h, int scan, const int *site_order, int nsites,
                              const int *bond_order, int nbonds, int on_device, int *first);

/* bs_perc's scan (Square/bs_perc.f:236-395) by O(N alpha) host replay:
   bonds bond_order[0..nbond) fixed, sites added in site_order; *first = the
   site count at which a cluster spans (0 if none).  c0_overflow != 0
   reproduces the flang-built reference, whose out-of-bounds read of c(0)
   exceeds every cluster size (hazard H11: a site whose first neighbour
   bond is unoccupied leaves the lattice together with every cluster it
   touches); c0_overflow == 0 is the intended site+bond connectivity. */
int perc_bs_perc_replay(int lattice, int m, int n, int pbc, const int *site_order, int nsites,
                        const int *bond_order, int nbond, int c0_overflow, int *first);

/* Same numbering without a context or device: host-only O(N alpha) replay
   of an explicit occupancy (used by the drivers' text output and tests).
   kind PERC_BONDSITE replays Square/bondsite.f:182-354 (bonds first, each a
   size-1 cluster, then sites merging their neighbour bonds' clusters; sizes
   count bonds and sites; spanning: lowest label of size >= 2n-1 holding a
   bottom- and a top-row site, bondsite.f:364-415).  csize needs
   cap >= t + nb + 2; stats = {cln, maxcn, maxcs, perccln}. */
int perc_replay_labels(int lattice, int m, int n, int pbc, int kind, int nsites,
                       const int *site_order, int nbonds, const int *bond_order,
                       int *bond_label, int *site_label, int *csize, int cap,
                       int *stats);
/* bondc.f's per-bond trace (bondocc.txt, Square/bondc.f:194-376): for the
   first nbond entries of bond_order (1-based ids, 0 = the spill slot),
   trace[3i] = 0 when the bond found no occupied neighbour bond and opened
   cluster trace[3i+1], 1 when it joined the largest neighbouring cluster
   trace[3i+1]; trace[3i+2] = that cluster's size after the step (host
   replay; the Fortran bondc driver writes bondocc.txt from it with
   trace = 1). */
int perc_replay_bond_trace(int lattice, int m, int n, int pbc, int nbond, const int *bond_order,
                           int *trace);
/* site.f's per-site trace (siteocc.txt, Square/site.f:167-272,
   Triangular/site.f): for the first nsite entries of site_order (1-based
   ids), PERC_SITE_TRACE ints each: [0] the site, [1..6] nearestn (scn
   used), [7] the neighbour with the largest cluster, [8] that cluster's
   number, [9] its size, [10] k = clusters absorbed, [11 + 2j] the size
   added and [12 + 2j] the largest cluster's size after (j < k), [21] the
   cluster the site joined, [22] its size after the step (host replay; the
   Fortran site driver writes siteocc.txt from it with trace = 1).
   PERC_EREPLAY for an id outside 1..m*n. */
#define PERC_SITE_TRACE 24
int perc_replay_site_trace(int lattice, int m, int n, int pbc, int nsite, const int *site_order,
                           int *trace);
/* The mixed programs' debug logs (sbdebug.txt, Square/sitebond.f:184-465;
   bsdebug.txt, Square/bondsite.f:178-418): the second phase's steps as an
   int stream, one record per order entry (host replay, kind PERC_SITEBOND
   or PERC_BONDSITE, the other arguments as perc_replay_labels).
   PERC_SITEBOND, per bond of bond_order[0..nbonds):
     {0, cln}                      both end sites empty: a new cluster
     {1, a, lcn, size}             only site a occupied, bond joins its cluster
     {2, b, lcn, size}             only site b occupied
     {3, a, la, ca, b, lb, cb, size}     both in one cluster
     {4|5, a, la, ca, b, lb, cb, ns, ns sites, nk, nk bond ids, lcn, size,
      oldcn}                       different clusters: 4 when a's is larger,
                                   5 otherwise; the sites and bonds (1-based
                                   list ids) relabelled oldcn -> lcn in index
                                   order; cluster oldcn is then empty
     {6}                           the shuffle's spill slot (0, 0)
   PERC_BONDSITE, per site of site_order[0..nsites):
     {0, cln}                      no occupied neighbour bond: a new cluster
     {1, k, k x (size added, largest cluster after), lcn, size}
   *len receives the stream length; trace may be NULL to size it, otherwise
   PERC_EINVAL when cap < *len. */
int perc_replay_mixed_trace(int lattice, int m, int n, int pbc, int kind, int nsites,
                            const int *site_order, int nbonds, const int *bond_order, int *trace,
                            long long cap, long long *len);

/* ---- conductance ----------------------------------------------------- */
typedef struct {
  double gtop, gbot;  /* Itop/Va, |Ibot|/Va                                  */
  double err;         /* final linbcg err                                    */
  int iter;           /* linbcg iterations                                   */
  int status;         /* 0 ok, 1 = no spanning cluster (G = 0)               */
  double t_assemble_ms, t_solve_ms, t_currents_ms;
} perc_cond_result;

/* Assemble the interior Kirchhoff system of the chosen spanning component
   (CSR, diagonal first), solve it with the fused Jacobi-PCG that follows
   linbcg's operation order and stopping rule (itol 1 or 2), and compute
   the terminal currents.  itol 3 / 4 (NR's step-size estimate in the L2 /
   max norm, bondc.f:816-832; the reference calls only itol 2) run a plain
   CSR PCG with per-iteration host folds; PERC_EITOL outside 1..4.
   vint_out (optional, host, t-2m doubles). */
int perc_conductance(perc_ctx *h, int rule, int cur_rule, double Va, double g0,
                     double leak, int itol, double tol, int itmax,
                     perc_cond_result *res, double *vint_out);

/* Matrix access for parity tests / roofline runs: copy the assembled
   interior CSR (0-based: rowptr[N+1], col[nnz], val[nnz], diag[N], rhs[N]).
   Pass NULL to skip an array; *nnz_out receives nnz. */
int perc_get_system(perc_ctx *h, int *rowptr, int *col, double *val,
                    double *diag, double *rhs, int *n_out, int *nnz_out);
/* y = A x on the assembled system (dsprsax order), host in / host out */
int perc_spmv_host(perc_ctx *h, const double *x, double *y);
/* Roofline probe: `reps` back-to-back launches of one solver kernel on the
   assembled system; returns mean kernel ms (HIP events on the context
   stream).  which: 0 = SpMV (dsprsax), 1 = CG SpMV + q.p dot, 2 = CG
   residual update (B), 3 = CG x/p update (P), 4 = STREAM copy 512 MB ->
   512 MB (16-B accesses, past the 256 MB Infinity Cache; the achievable-HBM
   reference), 5 = one whole CG iteration (every kernel of it, in order),
   6 = the resident solve's synchronisation floor: per iteration, the two
   block sums + grid all-gathers of k_cg_res on dummy values, nothing else
   (only on a context whose system takes the resident solver; else
   PERC_EHIP).  (Round 4 dropped the probes that lost their A/Bs: the
   16-B-entry CSR SpMV and the L = 8192 march geometries / load policies,
   profiles/r4_3_*.)  Clobbers solver vectors. */
int perc_bench_kernel(perc_ctx *h, int which, int reps, double *ms);
/* Self-test of the solver's table division (z = r/d from y = RN(1/d) and
   one Markstein correction, bitwise IEEE division when it holds) on the
   default device: n random (a, d) pairs; out3[0] = mismatches against `/`,
   out3[1..2] = bit patterns of the first mismatching a and d. */
int perc_selftest_division(long long n, unsigned long long seed, unsigned long long *out3);

/* Live kernel timing: when enabled, the CG launches of every 64th
   iteration (PERC_TIME_EVERY=n: every n-th) inside perc_conductance are
   bracketed by HIP events on the context stream (a timed launch opens a
   dispatch gap of several us: every 8th cost ~1 % of an L = 4096 solve,
   every launch ~10 %); the accumulated device time of the sampled launches
   that did work is returned (ms) with their count.  stats[0..5] = {spmv_ms, spmv_launches, resid_ms (B),
   resid_launches, xp_ms (P), xp_launches}; reset clears the accumulators. */
int perc_set_kernel_timing(perc_ctx *h, int enable);
int perc_kernel_stats(perc_ctx *h, double *stats, int reset);
/* Sizes of the assembled system: out[0] = N (rows), out[1] = nnz (off-diagonal) */
int perc_system_size(perc_ctx *h, long long *out);

/* Operator format of the solver.  The Kirchhoff matrix of a lattice has two
   distinct off-diagonal values (-g0 inside the spanning component, -leak
   elsewhere, bondc.f:482-538) on a fixed stencil, so besides the CSR copy
   the assembly writes a 16-bit code per row (bit j = "in" for the j-th
   sorted neighbour slot, slot count, row form) and the SpMV/CG kernels
   rebuild each row -- values, diagonal and summation order -- from that
   code: bitwise the same numbers as the CSR path from 2 of its 76 bytes.
   PERC_FMT_AUTO (default) uses the stencil operator whenever every stencil
   bond exists; the NR symbols (sprsin_/linbcg_) always use CSR.
   PERC_FMT_STENCIL fuses the p update into the SpMV: the register-march
   kernel when m is a multiple of 128, else the LDS-tiled one (m even). */
#define PERC_FMT_AUTO 0
#define PERC_FMT_CSR 1
#define PERC_FMT_STENCIL 2        /* stencil, p update fused into the SpMV  */
#define PERC_FMT_STENCIL_SPLIT 3  /* stencil, separate p-update and SpMV kernels */
#define PERC_FMT_STENCIL_TILED 4  /* stencil, fused, always the LDS-tiled kernel */
int perc_set_matrix_format(perc_ctx *h, int fmt);
/* Interior voltages.  linbcg never reads x inside its iteration and the
   terminal currents read it only on the interior rows next to the
   electrodes (Square/bondc.f:554-592), so perc_conductance keeps x on those
   2m rows only (bitwise the same values there) unless vint_out is given or
   this option is on -- then every row is updated every iteration, as
   linbcg does.  Default off. */
int perc_set_full_voltages(perc_ctx *h, int enable);

/* Row-slab decomposition of the CG solve (replaces
   one linbcg loop, Square/bondc.f:780-836): the interior rows split into
   nslab contiguous slabs with private r, p, q, x and one ghost row of r and
   p towards each neighbour; per iteration each slab runs the march P+S and
   the streaming B kernels on its rows, the q.p and z.r / r.r partials are
   combined in slab order, and the slabs' edge rows of r are copied into
   the neighbours' ghost rows.  Per-row arithmetic is the single-slab
   solve's; only the dot-product association differs.  Needs the register-
   march format (m a multiple of 128, PERC_FMT_STENCIL); a solve with
   nslab > 1 in another format fails with PERC_EHIP.  Default 1. */
int perc_set_slabs(perc_ctx *h, int nslab);

/* Distributed row slabs: one process per GPU solves slab s of K of the
   system assembled by perc_assemble (every process labels and assembles
   the whole lattice; the solve is split).  The per-slab kernels and the
   slab-order combine are perc_set_slabs's, so K processes reproduce its
   K-slab numbers bitwise.  The caller moves data between processes
   (percolation_amd/dslab.py: torch.distributed, RCCL on the context's
   stream or gloo through the host), through device buffers it owns:
     part_out  4 doubles   this slab's partials after a step (send);
     part_all  4K doubles  every slab's part_out in slab order (receive);
     edge_lo / edge_hi     m doubles: r of the slab's first / last row
                           (send to slab s-1 / s+1; NULL at s = 0 / K-1);
     ghost_lo / ghost_hi   m doubles: slab s-1's last / s+1's first row
                           (receive).
   Protocol: perc_dslab_begin (prologue; publishes part_out and the edges;
   the PS / B steps' kernels write their partials into part_out themselves)
   -> all-gather part_out into part_all, exchange edges into ghosts ->
   step COMBINE_INIT, GHOSTS; then per iteration: PS, all-gather,
   COMBINE_PS, B, all-gather, COMBINE_B, exchange edges, GHOSTS; poll
   perc_dslab_status every few iterations (the steps are no-ops once the
   stop test fired: every process takes the same decision).  perc_dslab_end
   puts this slab's x rows (the electrode rows unless full_x) into the
   context's x; perc_x_row / perc_currents then give Gtop / Gbot on the
   process that holds both electrode rows. */
typedef struct perc_dslab_bufs {
  double *part_out, *part_all, *edge_lo, *edge_hi, *ghost_lo, *ghost_hi;
} perc_dslab_bufs;
#define PERC_DSLAB_COMBINE_INIT 0
#define PERC_DSLAB_PS 1
#define PERC_DSLAB_COMBINE_PS 2
#define PERC_DSLAB_B 3
#define PERC_DSLAB_COMBINE_B 4
#define PERC_DSLAB_GHOSTS 5
int perc_dslab_begin(perc_ctx *h, int K, int s, int itol, double tol, int itmax, int full_x,
                     const perc_dslab_bufs *bufs);
int perc_dslab_step(perc_ctx *h, int op);
int perc_dslab_status(perc_ctx *h, int *iter, double *err, int *done);
int perc_dslab_end(perc_ctx *h);
/* The whole split solve from one host process, no caller code inside the
   loop: K labeled contexts (the same lattice and occupancy, context s on
   its own device for RCCL) solve row slab s each, one host thread per
   context issuing its slab's loop onto the context's stream.  xport
   PERC_XPORT_RCCL: ncclCommInitAll over the contexts' devices, the
   partials all-gathered and the r halo swapped by ncclAllGather /
   ncclSend / ncclRecv on the streams (no host round trip inside the loop);
   PERC_XPORT_HOST: the same exchanges staged through host memory (any
   devices, several contexts on one GPU included).  The numbers are
   perc_set_slabs(K)'s in one context bitwise.  Assembles every context
   (perc_assemble), solves, and returns Gtop / Gbot from slab 0 in *res
   (status 1: nothing spans).  Replaces the linbcg call of
   Fortran/Square/bondc.f:545 for a lattice split over GPUs.
   K = 1 runs the one-slab kernel epilogues (no combine, no collective: the
   same arithmetic) unless xport has PERC_XPORT_EXCHANGE set, which keeps
   the combines and the (one-rank) collectives -- the exchange machinery's
   own cost, measured by tools/dslab_bench.py.  RCCL communicators are made
   once per device list and kept for the process (one group call at a time
   per device list). */
#define PERC_XPORT_RCCL 0
#define PERC_XPORT_HOST 1
#define PERC_XPORT_EXCHANGE 4
int perc_dslab_solve_group(int K, perc_ctx **ctxs, int xport, int rule, int cur_rule, double Va,
                           double g0, double leak, int itol, double tol, int itmax, int full_x,
                           perc_cond_result *res);
/* One process per GPU (torchrun / MPI): rank 0 makes an RCCL unique id
   (PERC_DSLAB_ID_BYTES bytes), the launcher ships it to every rank, each
   rank binds its labeled context to slab s of K with perc_dslab_comm_init,
   then perc_dslab_solve runs the whole loop of perc_dslab_solve_group for
   its slab (assembly, all-gathers and halos over RCCL on the context's
   stream, the top electrode row to rank 0, rank 0's Gtop / Gbot broadcast
   to every rank).  The ranks check that they all found the same spanning
   state before the loop.  The communicator lives until perc_dslab_comm_free
   or perc_ctx_destroy.  Same numbers as perc_dslab_solve_group over K
   contexts. */
#define PERC_DSLAB_ID_BYTES 128
int perc_dslab_unique_id(void *id, int nbytes);
int perc_dslab_comm_init(perc_ctx *h, int K, int s, const void *id, int nbytes);
int perc_dslab_comm_free(perc_ctx *h);
int perc_dslab_solve(perc_ctx *h, int rule, int cur_rule, double Va, double g0, double leak,
                     int itol, double tol, int itmax, int full_x, perc_cond_result *res);
/* assembly only (perc_conductance's first half): the Kirchhoff system of
   the lowest spanning cluster; PERC_ESTATE before perc_label, status 1 in
   *spanning = 0 when nothing spans */
int perc_assemble(perc_ctx *h, int rule, double g0, double leak, double Va, int *spanning);
/* copy row `row` of the interior voltages between the context and a device
   buffer of m doubles (to_ctx = 1: into the context) */
int perc_x_row(perc_ctx *h, int row, double *dev_buf, int to_ctx);
/* terminal currents of the context's x (perc_conductance's last step) */
int perc_currents(perc_ctx *h, int rule, int cur_rule, double Va, double g0, double leak,
                  perc_cond_result *res);
/* the HIP stream the context enqueues on (hipStream_t), e.g. for a caller's
   collectives on the same stream */
void *perc_stream(perc_ctx *h);

/* Band height (lattice rows per wave) of the register-march kernel; 0 (default)
   picks the tallest of 32, 16, .. 2 rows that still gives >= 4096 waves.
   A tuning / test knob: results are the same up to the association of the
   q.p dot. */
int perc_set_march_rows(perc_ctx *h, int rows);

/* Register-march loop structure (PERC_FMT_STENCIL with m a multiple of
   128).  Per-row arithmetic is the same in every mode (bitwise the same
   values); only the association of the dot products differs.  The mode is
   read when the system is assembled; default PERC_MARCH_DEFAULT.
   PERC_MARCH_QFREE: the P+S kernel does not store q; the B kernel (r -= ak
   q, z.r, r.r) marches too and rebuilds q = A p(k) from p(k), so an
   iteration moves 52 instead of 60 bytes per row (strip-major at L = 4096:
   0.164 vs 0.178 ms per iteration; row-major at L = 8192: 0.721 vs 0.737).
   PERC_MARCH_ALT: neighbouring bands walk in opposite directions, so the
   halo rows they share are read at the same moment (cache hits).
   PERC_SOLVE_RESIDENT: the one-workgroup solve of small systems and the
   resident cooperative solve where they apply.
   PERC_MARCH_STRIPS (with QFREE): r, p and the row codes strip-major for the
   solve (each 128-column strip contiguous), so every wave walks one
   contiguous stream; x stays row-major.  Used while one vector fits the
   256 MB Infinity Cache (L <= 4096).
   PERC_MARCH_SLOTS: one workgroup per CU and round, the bands sized by the
   round a wave runs in (the first round on a CU streams fastest), so every
   wave finishes at about the same time (past the Infinity Cache: the
   row-major P kernel's one round of bands).
   PERC_MARCH_TAG (strip-major march): the end-of-kernel reductions publish
   tagged {value, tag} granules the readers poll for, instead of draining
   stores before each ticket; bitwise the same totals.
   PERC_MARCH_NIBBLE (strip-major march, square lattice): the row codes as
   one 4-bit slot mask per site (two sites per byte), count and form from
   the column -- 0.5 instead of 2 bytes of code per element in each kernel
   (52N -> 49N bytes per iteration); bitwise the same codes (checked per
   row when packed).
   Row slabs (perc_set_slabs) and the literal dot order always run the
   row-major q-storing march.  (Round 4 removed the variants that lost their
   A/Bs: workgroup row-march 4, deferred reductions 32, persistent march
   256, the strip-major march past the Infinity Cache 1024; those bits are
   rejected.) */
#define PERC_MARCH_QFREE 1
#define PERC_MARCH_ALT 2
#define PERC_SOLVE_RESIDENT 8
#define PERC_MARCH_STRIPS 16
#define PERC_MARCH_SLOTS 64
#define PERC_MARCH_TAG 128
#define PERC_MARCH_NIBBLE 512
#define PERC_MARCH_DEFAULT                                                                      \
  (PERC_MARCH_QFREE | PERC_MARCH_ALT | PERC_SOLVE_RESIDENT | PERC_MARCH_STRIPS | PERC_MARCH_SLOTS | \
   PERC_MARCH_TAG | PERC_MARCH_NIBBLE)
int perc_set_march_mode(perc_ctx *h, int mode);
/* Per-round band weights of the slot-weighted bands (PERC_MARCH_SLOTS):
   which = 0 the strip-major P kernel, 1 its B kernel, 2 the row-major P past
   the Infinity Cache; n = 0 restores every default (100:75:50, 100:80:60,
   flat).  A tuning / test knob: the rows stay a partition of the lattice
   whatever the weights. */
int perc_set_band_weights(perc_ctx *h, int which, int n, const int *w);

/* Association of linbcg's three dot products (Square/bondc.f:785-787 bknum,
   :803-805 akden, :872-875 snrm).  PERC_DOT_FAST (default): deterministic
   wave / workgroup trees inside the fused kernels.  PERC_DOT_LITERAL: each
   sum folded term after term in ascending j on one wave of the GPU, exactly
   as the reference loops do -- with every other operation already the
   reference's, the iterates, iter, err history and voltages are then
   bitwise the reference solver's.  One dependent fp64 add per term: a
   verification mode (single slab).  It runs the production kernels of the
   fast order -- the q-free strip-major / row-major march (k_cg_march P, B)
   and the resident solve (k_cg_res), the same code objects -- which store
   each row's dot terms (the reference's IEEE products) for the folds; other
   formats fold from their stored q, p, r.  perc_last_solve says what ran.
   The NR drop-in linbcg_ uses PERC_DOT_LITERAL by default
   (perc_nr_set_dot_order). */
#define PERC_DOT_FAST 0
#define PERC_DOT_LITERAL 1
/* PERC_DOT_LITERAL_HOST: the literal order with the three serial sums formed
   by the host CPU from the terms the q-free march kernels stored (the same
   IEEE adds in the same ascending-j order, so bitwise PERC_DOT_LITERAL; the
   CPU's dependent fp64 add is ~4x shorter than a GPU wave's, which makes the
   config-size verification runs fit one GPU session).  Runs the launched
   march (not the resident solve); formats without it fold on the GPU. */
#define PERC_DOT_LITERAL_HOST 2
int perc_set_dot_order(perc_ctx *h, int order);
/* What the last solve of the context actually ran: out4[0] = kernel family
   (0 other launched kernels: LDS tiles, split stencil, CSR; PERC_RAN_MARCH,
   PERC_RAN_RESIDENT, PERC_RAN_SMALL), out4[1] = PERC_RAN_* flag bits,
   out4[2] = iterations, out4[3] = 0 (reserved).  PERC_ESTATE before any
   solve. */
#define PERC_RAN_MARCH 1
#define PERC_RAN_SLABS 2      /* row slabs (perc_set_slabs) */
#define PERC_RAN_RESIDENT 3
#define PERC_RAN_SMALL 4
#define PERC_RAN_LITERAL 1    /* literal dot order */
#define PERC_RAN_LIT_TERMS 2  /* ... folding the terms the solve kernels stored */
#define PERC_RAN_QFREE 4      /* q-free march (P + B rebuild q) */
#define PERC_RAN_STRIPS 8     /* strip-major layout */
#define PERC_RAN_NIBBLE 16    /* 4-bit row codes */
#define PERC_RAN_TAG 32       /* tagged-granule reductions */
#define PERC_RAN_HOST_FOLD 64 /* PERC_DOT_LITERAL_HOST: the sums folded by the host */
#define PERC_RAN_XCD_GROUPED 128 /* resident solve: XCD-grouped reductions (else the flat all-gather) */
#define PERC_RAN_DEFERRED 256 /* march: each launch's totals formed by the next launch (no collector tail) */
int perc_last_solve(perc_ctx *h, int *out4);
/* err of every iteration of the last solve (linbcg's per-iteration
   `write (*,*) iter, err`, bondc.f:834): min(cap, iterations) values into
   out, entry k - 1 = err of iteration k; returns the iteration count (>= 0)
   or a negative status.  itol 3 / 4: EVERY iteration has its entry, also
   those where linbcg takes `goto 100` (bondc.f:822-831) and prints nothing;
   there the entry is the err linbcg set before the jump, znrm / bnrm -- so
   the history has more entries than the reference's log, which holds only
   the tested iterations.  itol 1 / 2: entry for entry the reference's log. */
int perc_err_history(perc_ctx *h, double *out, int cap);
/* Random bond conductances (MATLAB/ConductCalc.m condtype 2, :38-47 and
   :94-97): the bonds of the spanning cluster get G = -g0 * w[id] instead of
   -g0 (w[id] = the MATLAB rand drawn for that bond; the draw order is the
   caller's, see api.conductcalc_weights).  w = NULL restores fixed
   conductances.  n = the lattice's bond count.  With weights the solver
   runs the CSR operator (the stencil code encodes two values only). */
int perc_set_bond_weights(perc_ctx *h, const double *w, long long n);
/* ConductCalc.m condtype 2 from C / Fortran (MATLAB/ConductCalc.m:38-47,
   94-97, 114-118, 136-146): after perc_label, every bond the assembly gives
   -g0 under `rule` (the spanning cluster's) gets -g0*rand, one
   rand('twister', seed) draw per such bond in bond-list order; the others
   keep their value (perc_set_bond_weights with those multipliers; no
   spanning cluster: fixed conductances).  perc_twister_uniform: n draws of
   that generator (MT19937 init_genrand(seed), 53-bit genrand_res53
   doubles).  MATLAB parity itself is unpinned (no MATLAB here). */
int perc_set_conductcalc_weights(perc_ctx *h, int rule, unsigned int seed);
int perc_twister_uniform(unsigned int seed, long long n, double *out);
/* Solver loop of the assembled system: out5[0] = 0 (no march kernel: LDS
   tiles, split or CSR), 1 (per-wave march k_cg_march), 3 (resident
   persistent solve k_cg_res), 4 (one-workgroup solve of a small system,
   k_cg_small: N <= 8192 under PERC_FMT_AUTO with PERC_SOLVE_RESIDENT set);
   out5[1] = bit 0: q-free B, bit 1: strip-major solve layout, bit 3:
   slot-weighted bands (PERC_MARCH_SLOTS; past the Infinity Cache the
   row-major P kernel's one round of bands), bit 4: tagged-granule
   reductions, bit 5: nibble row codes (the last solve); out5[2] = alternating directions, out5[3] = band height,
   out5[4] = strip width (columns). */
int perc_march_info(perc_ctx *h, int *out5);

/* format the solver kernels use on the assembled system: PERC_FMT_CSR,
   PERC_FMT_STENCIL (register-march fused kernel), PERC_FMT_STENCIL_TILED
   (LDS-tiled fused kernel) or PERC_FMT_STENCIL_SPLIT */
int perc_matrix_format(perc_ctx *h);

/* ---- one hot-path realisation (bench / ensemble) ---------------------- */
typedef struct {
  perc_label_info label;
  perc_cond_result cond;
  double t_upload_ms, t_label_ms, t_total_ms;
} perc_realisation;
/* occupy + label + conductance for PERC_BOND with the bondc rules;
   bond_order is a host array, or a device array when on_device != 0 */
int perc_bondc_realisation(perc_ctx *h, int tbonds, const int *bond_order,
                           int on_device, double Va, double g0, double tol,
                           int itmax, perc_realisation *out);

/* ---- ensemble statistics (bond_cond, config 4) ----------------------- */
/* Accumulate stats for one pb point: {count, sum G, sum G^2, count spanning,
   sum iter} into acc[5*point..]. */
void perc_stats_accumulate(double *acc, int point, double g, int spanning, int iter);

/* ---- multi-GPU ensemble (one process, one host thread per device) ----- *
 * Replaces the reference's serial trial loop (Fortran/Square/bond_cond.f:
 * 62-70 seeds, :123-498 trials, rows written at :481-482).  Trial ii
 * (1-based) runs on device (ii-1) mod ndev; each device has its own
 * perc_ctx and host thread; per-trial results land in the caller's arrays
 * at index ii-1 (ii order whatever device ran them).  The only collective
 * is one RCCL all-reduce (sum, fp64) over a communicator ncclCommInitAll
 * builds across the devices. */
typedef struct perc_ensemble perc_ensemble;
/* devices == NULL: devices 0..ndev-1 */
int perc_ensemble_create(int ndev, const int *devices, int lattice, int m, int n, int pbc,
                         perc_ensemble **out);
int perc_ensemble_destroy(perc_ensemble *e);
int perc_ensemble_ndev(perc_ensemble *e);
/* W (1..64) contexts, host threads and streams per device for the trial
   loops (default 1): trial ii runs on device (ii-1) mod ndev and there on
   worker ((ii-1) / ndev) mod W; per-trial results are the same, the
   per-device statistics are summed over the workers in worker order before
   the all-reduce.  For small lattices, whose trials leave a device mostly
   idle.  perc_ensemble_workers returns W. */
int perc_ensemble_set_workers(perc_ensemble *e, int workers);
int perc_ensemble_workers(perc_ensemble *e);
/* device dev's own context (e.g. for single-trial calls); NULL if out of range */
perc_ctx *perc_ensemble_ctx(perc_ensemble *e, int dev);
/* the trials device `dev` of `ndev` runs, 1-based, ascending (ii_out may be
   NULL); returns their count.  Host-only. */
int perc_ensemble_trials(int ntrials, int ndev, int dev, int *ii_out);
/* stats holds ndev slices of k doubles (device d's at stats[d*k]); on return
   every slice holds the element-wise sum over the devices (ncclAllReduce). */
int perc_ensemble_allreduce(perc_ensemble *e, double *stats, int k);
/* bond_cond over the devices: trial ii shuffles with tseed[ii-1] (tseed must
   hold at least ntrials seeds; the reference's tseed(1000) caps numtrials at
   1000, bond_cond.f:62-70, callers extend the stream past it) (REAL*4
   Fisher-Yates, bondc.f:162-174), computes the lowest-label conductance at
   grid points nbarr[0..) until a value <= 0, a repeat (hazard H3) or npts;
   outputs, per trial t = ii-1: nrows[t] rows at [t*npts + j] of gbot, gtop,
   iters; bf_c[t] = first spanning bond count (0: none), perccln[t] = lowest
   spanning label with every bond occupied (bond_cond.f:381, 486-496).
   stats (npts*5, may be NULL) = the all-reduced {count, sum Gtop,
   sum Gtop^2, count spanning, sum iter} per grid point. */
int perc_ensemble_bond_cond(perc_ensemble *e, int ntrials, const int *tseed, int npts,
                            const int *nbarr, double Va, double g0, double tol, int itmax,
                            int *nrows, double *gbot, double *gtop, int *iters, int *bf_c,
                            int *perccln, double *stats);
/* REAL*4 Fisher-Yates of ids 1..N after srand(seed) on a stream local to the
   call (thread-safe; same sequence as perc_srand + perc_shuffle): order has
   N+1 slots, order[N] = 0 (hazard H2). */
void perc_shuffle_seeded(int seed, int N, int *order);

/* ---- Numerical-Recipes-compatible layer (F77 ABI, by reference) ------- *
 * Same names and argument meaning as the routines embedded in the
 * reference (Square/bondc.f:723-917).  linbcg_/atimes_/asolve_ read the
 * matrix from COMMON /mat/ sa(NMAX), ija(NMAX) (symbol mat_, NMAX=20000 as
 * in the reference) unless perc_nr_bind() points them at other storage.
 * linbcg_ runs the HIP PCG on device 0.  Errors that `pause` in the
 * reference are reported through perc_nr_status(). */
void sprsin_(double *a, int *n, int *np, double *thresh, int *nmax, double *sa, int *ija);
void dsprsax_(double *sa, int *ija, double *x, double *b, int *n);
void dsprstx_(double *sa, int *ija, double *x, double *b, int *n);
void atimes_(int *n, double *x, double *r, int *itrnsp);
void asolve_(int *n, double *b, double *x, int *itrnsp);
double snrm_(int *n, double *sx, int *itol);
void linbcg_(int *n, double *b, double *x, int *itol, double *tol, int *itmax,
             int *iter, double *err);
void perc_nr_bind(double *sa, int *ija, int nmax);
int perc_nr_status(void);
int perc_nr_status_(void);  /* F77 spelling: `integer perc_nr_status` */
/* association of linbcg_'s dot products (PERC_DOT_LITERAL by default: the
   NR drop-in reproduces the reference solver bitwise; PERC_DOT_FAST: the
   wave-tree sums of perc_conductance) */
int perc_nr_set_dot_order(int order);
/* call nearestn(rn) (Square/bondc.f:617-715, Triangular/bondc.f:619-804):
   the neighbours of site rn into the caller's blank COMMON m, n, t, pbc,
   nn(10), scn (symbol __BLNK__; scn 4 square, 6 triangular), zeros where a
   neighbour is missing; perc_nr_status() = PERC_ESTATE without one. */
void nearestn_(const int *rn);

#ifdef __cplusplus
}
#endif
#endif /* PERC_H */
