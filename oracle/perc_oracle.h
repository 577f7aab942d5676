/*
 * perc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference (IsaiahSteinke/Percolation, Fortran 77)
 * cluster-labeling + Kirchhoff-conductance path.  Only tests/, the smoke()
 * check in __graft_entry__.py and bench.py's cpu_baseline leg may load this
 * library; the product (libperc) never links or calls it.
 *
 * Parity pin: every function below is checked by tests/test_oracle_golden.py
 * against fixtures produced by the compiled reference Fortran (oracle/_ref,
 * built by oracle/build_ref.sh from /root/reference sources) and, for the RNG,
 * against libgfortran's own _gfortran_rand.  MATLAB ConductCalc.m rules
 * (site / mixed conductance) cannot be run here (no MATLAB): those are
 * "parity unpinned" and cross-checked by a direct sparse solve only.
 *
 * Conventions follow the reference: site ids 1..t row-major from the bottom
 * row, bonds (b1<b2) in bond-list order, arrays passed 0-based in C (element
 * k-1 holds Fortran index k).
 */
#ifndef PERC_ORACLE_H
#define PERC_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG: libgfortran rand/srand (Park-Miller 16807 mod 2^31-1) ---------- */
void or_srand(int seed);
float or_rand(int i);
int or_rng_state(void);

/* ---- lattice --------------------------------------------------------- */
/* lattice: 0 = square (scn 4, bcn 6), 1 = triangular (scn 6, bcn 10) */
int or_scn(int lattice);
int or_bcn(int lattice);
int or_nbonds(int lattice, int m, int n, int pbc);
/* nearestn(rn): fills nn[0..scn-1], zeros where no neighbour.
   Square/bondc.f:617-715, Triangular/bondc.f:619-804. */
void or_nearestn(int lattice, int m, int n, int pbc, int rn, int *nn);
/* bond list (Square/bondc.f:137-154): returns count written */
int or_bond_list(int lattice, int m, int n, int pbc, int *b1, int *b2);

/* ---- occupation order (float32 Fisher-Yates, Square/bondc.f:162-174) --- */
/* o1,o2 have nb+1 slots; slot nb (0-based) must be zero on entry (H2). */
void or_shuffle_pairs(int nb, int *o1, int *o2);
/* order has t+1 slots, slot t zero (Square/site.f:139-147) */
void or_shuffle_ints(int t, int *order);
/* tseed(1..k) from master seed (Square/bond_cond.f:65-70) */
void or_trial_seeds(int master, int k, int *tseed);

/* ---- labeling (literal O(N^2) restatement of the reference loops) ------ */
/* bond percolation: Square/bondc.f:189-393.  label[nb] (b(:,3)), csize[cap]
   (c(:), cap >= nb+2), returns cln (next unused label); maxcn/maxcs out.
   o1/o2: order (nb+1 slots).  tbonds bonds are occupied. */
int or_label_bonds_literal(int lattice, int m, int n, int pbc, int nb,
                           const int *b1, const int *b2,
                           const int *o1, const int *o2, int tbonds,
                           int *label, int *csize, int *maxcn, int *maxcs);
/* same semantics, union-find replay (O(N alpha)) */
int or_label_bonds_replay(int lattice, int m, int n, int pbc, int nb,
                          const int *b1, const int *b2,
                          const int *o1, const int *o2, int tbonds,
                          int *label, int *csize, int *maxcn, int *maxcs);
/* site percolation: Square/site.f:162-289.  s[t], csize[cap>=t+2] */
int or_label_sites_literal(int lattice, int m, int n, int pbc,
                           const int *order, int tsites,
                           int *s, int *csize, int *maxcn, int *maxcs);
int or_label_sites_replay(int lattice, int m, int n, int pbc,
                          const int *order, int tsites,
                          int *s, int *csize, int *maxcn, int *maxcs);
/* mixed site-then-bond: Square/sitebond.f:187-400 (literal). */
int or_label_sitebond(int lattice, int m, int n, int pbc, int nb,
                      const int *b1, const int *b2,
                      const int *sorder, int tsites,
                      const int *o1, const int *o2, int tbonds,
                      int *s, int *blabel, int *csize, int *maxcn, int *maxcs);

/* same, union-find replay (O(N alpha)); csize cap >= t + nb + 2 */
int or_label_sitebond_replay(int lattice, int m, int n, int pbc, int nb,
                             const int *b1, const int *b2,
                             const int *sorder, int tsites,
                             const int *o1, const int *o2, int tbonds,
                             int *s, int *blabel, int *csize, int *maxcn, int *maxcs);
/* canonical partition ids (min site of the cluster; 0 = no cluster) */
void or_canon_sites(int t, const int *s, int maxlab, int *canon);
void or_canon_bonds(int t, int nb, const int *b1, const int *b2, const int *label, int maxlab,
                    int *canon);

/* mixed bonds-then-sites: Square/bondsite.f:170-322 (literal); border =
   bond ids (0: spill slot), s[t], blabel[nb], csize[t+nb+2]; returns cln */
int or_label_bondsite(int lattice, int m, int n, int pbc, int nb,
                      const int *b1, const int *b2,
                      const int *border, int tbonds,
                      const int *sorder, int tsites,
                      int *s, int *blabel, int *csize, int *maxcn, int *maxcs);

/* ---- spanning detection --------------------------------------------- */
/* bond: lowest label l < cln with c(l) >= n-1 touching bottom (b1<=m) and
   top (b2>t-m) (Square/bondc.f:413-456).  0 if none. */
int or_span_bonds(int m, int n, int nb, const int *b1, const int *b2,
                  const int *label, const int *csize, int cln);
/* site: c(l) >= n, s(j)=l for some j<=m and some j>t-m (Square/site.f:309-344)
   mixed: minsize = 2n-1 (Square/sitebond.f:423-458) */
int or_span_sites(int m, int n, const int *s, const int *csize, int cln,
                  int minsize);

/* ---- conductance ----------------------------------------------------- */
/* per-bond conductance-matrix entry rules (all return G(b1,b2), negative) */
/* rule 0 bond (bondc.f:482-489), 1 site (ConductCalc.m:88-102),
   2 mixed (ConductCalc.m:134-153) */
void or_bond_values(int rule, int nb, const int *b1, const int *b2,
                    const int *blabel, const int *s, int perccln, double g0,
                    double leak, double *gval);
/* Assembly (bondc.f:482-538): interior NR row-indexed storage (sprsin,
   thresh) + RHS Itemp + full diagonal.  sa/ija sized >= nmax (1-based NR
   layout in 0-based C arrays: sa[0] is sa(1)).  rhs_rule 0: Fortran
   Itemp - G*Va, 1: MATLAB Itemp + (-G)*Va.  Returns nnz used (k) or -1. */
int or_assemble(int lattice, int m, int n, int pbc, int nb, const int *b1,
                const int *b2, const double *gval, double Va, double thresh,
                int rhs_rule, int nmax, double *sa, int *ija, double *itemp,
                double *diag_full);
/* NR routines, literal (bondc.f:723-917) */
void or_dsprsax(const double *sa, const int *ija, const double *x, double *b,
                int n);
void or_dsprstx(const double *sa, const int *ija, const double *x, double *b,
                int n);
/* linbcg on (sa,ija); prints nothing; returns iter, err.  iter_err (optional,
   may be NULL) receives err per iteration (length >= itmax+1). */
void or_linbcg(const double *sa, const int *ija, int n, const double *b,
               double *x, int itol, double tol, int itmax, int *iter,
               double *err, double *iter_err);
/* the same iterates (itol 2) on a bitwise-symmetric sa, threaded, with
   snapshots of x (check_x[c*n..]) at the first iteration where err <=
   check_tols[c] (descending; the last one stops the run).  -1 if sa is not
   bitwise symmetric (see perc_oracle.c). */
int or_linbcg_sym(const double *sa, const int *ija, int n, const double *b,
                  double *x, int itmax, int nthreads, int ncheck,
                  const double *check_tols, double *check_x, int *check_iter,
                  double *check_err, int *iter_o, double *err_o,
                  double *iter_err, int dot_order);
/* Terminal currents (bondc.f:554-592): V from Vint; full-G sprsin with
   thresh (1e-10 in Fortran; 0 in MATLAB) restricted to the 2m boundary rows.
   cur_rule 0: Fortran (Ibot, Itop ascending), 1: MATLAB (Itop summed t..t-m+1)*/
void or_currents(int lattice, int m, int n, int pbc, int nb, const int *b1,
                 const int *b2, const double *gval, const double *diag_full,
                 const double *vint, double Va, double thresh, int cur_rule,
                 double *gtop, double *gbot);

/* one whole bondc realisation (labeling + spanning + conductance) */
typedef struct {
  int nb, tbonds, cln, maxcn, maxcs, perccln, perccls, iter;
  double gtop, gbot, err;
} or_bondc_result;
int or_bondc(int lattice, int m, int n, int pbc, double pb, int seed,
             double Va, double g0, int itmax, double tol, int literal,
             int *label_out, int *csize_out, int *o1_out, int *o2_out,
             or_bondc_result *res);

/* one bond_cond trial; rows sized >= 250.  Returns rows written. */
int or_bond_cond_trial(int lattice, int m, int n, int pbc, int tseed,
                       double Va, double g0, int itmax, double tol,
                       double *row_pb, double *row_gbot, double *row_gtop,
                       int *row_iter, int *perccln_out, double *pc_out);

#ifdef __cplusplus
}
#endif
#endif
