/*
 * perc_oracle.c -- TEST INFRASTRUCTURE ONLY (see perc_oracle.h).
 *
 * Plain-C restatement of the reference algorithm.  Each function cites the
 * reference file:line (paths relative to the reference root) it follows.
 * Compiled with -O2 -ffp-contract=off (no FMA contraction, IEEE float32 /
 * float64 semantics like the flang -O2 x86-64 reference build).
 */
#include "perc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================
 * RNG.  GNU Fortran runtime rand/srand (libgfortran intrinsics/rand.c,
 * GCC 7.5 as shipped in /opt/conda/lib/libgfortran.so.4): Park-Miller
 * minimal standard, a=16807, m=2^31-1; seed 0 -> 123459876; rand returns
 * ((x-1) & ~0x1FF) / 2^31 as REAL*4.  Call sites: Square/bondc.f:162,167,
 * Square/bond_cond.f:66-70,181-186, Square/site.f:131-147.
 * ==================================================================== */
static unsigned long long g_rand_seed = 1ULL;

static void srand_internal(long long i) {
  g_rand_seed = i ? (unsigned long long)i : 123459876ULL;
}
void or_srand(int seed) { srand_internal(seed); }
int or_rng_state(void) { return (int)g_rand_seed; }

static int irand_internal(int i) {
  switch (i) {
    case 0: break;
    case 1: srand_internal(0); break;
    default: srand_internal(i); break;
  }
  g_rand_seed = (16807ULL * g_rand_seed) % 2147483647ULL;
  return (int)g_rand_seed;
}

float or_rand(int i) {
  unsigned int mask = ~0u << 9; /* 32 - 24 + 1 */
  unsigned int v = ((unsigned int)(irand_internal(i) - 1)) & mask;
  return (float)v / (float)2147483646; /* (float)(2^31-2) == 2^31 */
}

/* ======================================================================
 * Lattice topology: nearestn.  Square/bondc.f:617-715 (square),
 * Triangular/bondc.f:619-804 (triangular "brick" layout, column parity).
 * nn[0..scn-1] receives the neighbours in reference order; 0 = none.
 * ==================================================================== */
int or_scn(int lattice) { return lattice ? 6 : 4; }
int or_bcn(int lattice) { return lattice ? 10 : 6; }

int or_nbonds(int lattice, int m, int n, int pbc) {
  /* Square/bondc.f:119-123, Triangular/bondc.f:121-125 */
  if (lattice == 0) return pbc ? m * (2 * n - 1) : 2 * m * n - m - n;
  return pbc ? m * (3 * n - 2) : 3 * m * n - 2 * m - 2 * n + 1;
}

static int fmod_(int a, int b) { return a % b; } /* Fortran MOD == C % */

static void nn_square(int m, int n, int pbc, int rn, int *nn) {
  int t = m * n;
  nn[0] = nn[1] = nn[2] = nn[3] = 0;
  if (rn == 1) { nn[0] = rn + 1; nn[1] = rn + m; if (pbc) nn[2] = m; return; }
  if (rn == m) { nn[0] = rn - 1; nn[1] = rn + m; if (pbc) nn[2] = 1; return; }
  if (rn == t - (m - 1)) {
    nn[0] = rn - m; nn[1] = rn + 1; if (pbc) nn[2] = t; return;
  }
  if (rn == t) { nn[0] = rn - m; nn[1] = rn - 1; if (pbc) nn[2] = rn - (m - 1); return; }
  if (rn < m) { nn[0] = rn - 1; nn[1] = rn + 1; nn[2] = rn + m; return; }
  if (rn > t - m) { nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + 1; return; }
  if (fmod_(rn - 1, m) == 0) {
    nn[0] = rn - m; nn[1] = rn + 1; nn[2] = rn + m;
    if (pbc) nn[3] = rn + (m - 1);
    return;
  }
  if (fmod_(rn, m) == 0) {
    nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + m;
    if (pbc) nn[3] = rn - (m - 1);
    return;
  }
  nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + 1; nn[3] = rn + m;
}

static void nn_tri(int m, int n, int pbc, int rn, int *nn) {
  int t = m * n, z;
  for (z = 0; z < 6; z++) nn[z] = 0;
  /* lower-left corner */
  if (rn == 1) {
    nn[0] = rn + 1; nn[1] = rn + m; nn[2] = rn + (m + 1);
    if (pbc) { nn[3] = rn + (m - 1); nn[4] = rn + (2 * m - 1); }
    return;
  }
  /* lower-right corner */
  if (rn == m) {
    nn[0] = rn - 1; nn[1] = rn + m;
    if (fmod_(m, 2) == 1) { nn[2] = rn + (m - 1); return; }
    if (pbc) nn[2] = 1;
    return;
  }
  /* upper-left corner */
  if (rn == t - (m - 1)) {
    nn[0] = rn - m; nn[1] = rn + 1;
    if (pbc) nn[2] = t;
    return;
  }
  /* upper-right corner */
  if (rn == t) {
    if (fmod_(m, 2) == 1) { nn[0] = rn - m; nn[1] = rn - 1; return; }
    nn[0] = rn - (m + 1); nn[1] = rn - m; nn[2] = rn - 1;
    if (pbc) { nn[3] = rn - (2 * m - 1); nn[4] = rn - (m - 1); }
    return;
  }
  /* bottom row */
  if (rn < m) {
    if (fmod_(rn, 2) == 0) {
      nn[0] = rn - 1; nn[1] = rn + 1; nn[2] = rn + m;
    } else {
      nn[0] = rn - 1; nn[1] = rn + 1; nn[2] = rn + (m - 1); nn[3] = rn + m;
      nn[4] = rn + (m + 1);
    }
    return;
  }
  /* top row */
  if (rn > t - m) {
    if (fmod_(rn, 2) == 0) {
      nn[0] = rn - (m + 1); nn[1] = rn - m; nn[2] = rn - (m - 1);
      nn[3] = rn - 1; nn[4] = rn + 1;
    } else {
      nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + 1;
    }
    return;
  }
  /* left edge */
  if (fmod_(rn - 1, m) == 0) {
    nn[0] = rn - m; nn[1] = rn + 1; nn[2] = rn + m; nn[3] = rn + (m + 1);
    if (pbc) { nn[4] = rn + (m - 1); nn[5] = rn + (2 * m - 1); }
    return;
  }
  /* right edge */
  if (fmod_(rn, m) == 0) {
    if (fmod_(m, 2) == 1) {
      nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + (m - 1); nn[3] = rn + m;
      return;
    }
    nn[0] = rn - (m + 1); nn[1] = rn - m; nn[2] = rn - 1; nn[3] = rn + m;
    if (pbc) { nn[4] = rn - (2 * m - 1); nn[5] = rn - (m - 1); }
    return;
  }
  /* interior */
  {
    int up; /* 1: (rn-(m+1), rn-m, rn-(m-1), rn-1, rn+1, rn+m) form */
    if (fmod_(m, 2) == 1) {
      if (fmod_(rn / m, 2) == 0) up = (fmod_(rn, 2) == 0);
      else up = (fmod_(rn, 2) != 0);
    } else {
      up = (fmod_(rn, 2) == 0);
    }
    if (up) {
      nn[0] = rn - (m + 1); nn[1] = rn - m; nn[2] = rn - (m - 1);
      nn[3] = rn - 1; nn[4] = rn + 1; nn[5] = rn + m;
    } else {
      nn[0] = rn - m; nn[1] = rn - 1; nn[2] = rn + 1;
      nn[3] = rn + (m - 1); nn[4] = rn + m; nn[5] = rn + (m + 1);
    }
  }
}

void or_nearestn(int lattice, int m, int n, int pbc, int rn, int *nn) {
  if (lattice == 0) nn_square(m, n, pbc, rn, nn);
  else nn_tri(m, n, pbc, rn, nn);
}

int or_bond_list(int lattice, int m, int n, int pbc, int *b1, int *b2) {
  /* Square/bondc.f:137-154 */
  int t = m * n, scn = or_scn(lattice), rc = 0, i, j, nn[6];
  for (i = 1; i <= t - 1; i++) {
    or_nearestn(lattice, m, n, pbc, i, nn);
    for (j = 0; j < scn; j++) {
      if (nn[j] > i) { b1[rc] = i; b2[rc] = nn[j]; rc++; }
    }
  }
  return rc;
}

/* ======================================================================
 * Occupation order: REAL*4 Fisher-Yates (Square/bondc.f:166-174,
 * Square/site.f:139-147).  j = i + (N-i+1)*rand(0) evaluated in float32
 * and truncated (hazard H2: j may be N+1 -> zeroed slot N+1).
 * ==================================================================== */
static int fy_index(int i, int N) {
  float r = or_rand(0);
  float prod = (float)(N - i + 1) * r;
  float s = (float)i + prod;
  return (int)s;
}

void or_shuffle_pairs(int nb, int *o1, int *o2) {
  int i;
  for (i = 1; i <= nb; i++) {
    int j = fy_index(i, nb), t1, t2;
    if (j < 1) j = 1;           /* never observed; keeps the C array in bounds */
    if (j > nb + 1) j = nb + 1;
    t1 = o1[i - 1]; t2 = o2[i - 1];
    o1[i - 1] = o1[j - 1]; o2[i - 1] = o2[j - 1];
    o1[j - 1] = t1; o2[j - 1] = t2;
  }
}

void or_shuffle_ints(int t, int *order) {
  int i;
  for (i = 1; i <= t; i++) {
    int j = fy_index(i, t), tmp;
    if (j < 1) j = 1;
    if (j > t + 1) j = t + 1;
    tmp = order[i - 1]; order[i - 1] = order[j - 1]; order[j - 1] = tmp;
  }
}

void or_trial_seeds(int master, int k, int *tseed) {
  /* Square/bond_cond.f:65-70: tseed(i) = int(rand(0)*10000000)+1 */
  int i;
  or_srand(master);
  for (i = 0; i < k; i++) {
    float v = or_rand(0) * (float)10000000;
    tseed[i] = (int)v + 1;
  }
}

/* ======================================================================
 * Bond labeling, literal.  Square/bondc.f:194-393 (identical loop in
 * Square/bond_cond.f:200-348 and the triangular files).  c(0) is read when
 * a neighbour bond is empty (hazard H1); it is 0 here.
 * ==================================================================== */
/* one occupation step of the literal loop; state lives in the caller */
typedef struct {
  int lattice, m, n, pbc, nb, scn, bcn;
  const int *b1, *b2;
  int *label, *csize;
  int cln, maxcn, maxcs;
} lit_state;

static void lit_add_bond(lit_state *S, int a, int bb) {
  int j, k, l, nn[6], nnb[25][4], rc = 0, lcn, lcs, clsum;
  const int *b1 = S->b1, *b2 = S->b2;
  int *label = S->label, *csize = S->csize;
  memset(nnb, 0, sizeof(nnb));
  or_nearestn(S->lattice, S->m, S->n, S->pbc, a, nn);
  for (j = 0; j < S->scn; j++) {
    if (nn[j] != 0 && nn[j] != bb) {
      if (nn[j] > a) { nnb[rc][0] = a; nnb[rc][1] = nn[j]; }
      else { nnb[rc][0] = nn[j]; nnb[rc][1] = a; }
      rc++;
    }
  }
  or_nearestn(S->lattice, S->m, S->n, S->pbc, bb, nn);
  for (j = 0; j < S->scn; j++) {
    if (nn[j] != 0 && nn[j] != a) {
      if (nn[j] > bb) { nnb[rc][0] = bb; nnb[rc][1] = nn[j]; }
      else { nnb[rc][0] = nn[j]; nnb[rc][1] = bb; }
      rc++;
    }
  }
  for (j = 0; j < S->nb; j++)
    for (k = 0; k < S->bcn; k++)
      if (b1[j] == nnb[k][0] && b2[j] == nnb[k][1]) {
        nnb[k][2] = label[j];
        nnb[k][3] = csize[label[j]];
      }
  lcn = nnb[0][2];
  lcs = nnb[0][3];
  for (k = 1; k < S->bcn; k++)
    if (nnb[k][0] != 0 && nnb[k][2] != 0 && nnb[k][3] > lcs) {
      lcn = nnb[k][2];
      lcs = nnb[k][3];
    }
  if (lcs == 0) {
    for (j = 0; j < S->nb; j++)
      if (b1[j] == a && b2[j] == bb) label[j] = S->cln;
    csize[S->cln] = 1;
    S->cln++;
  } else {
    clsum = lcs;
    for (k = 0; k < S->bcn; k++) {
      if (nnb[k][0] != 0 && nnb[k][2] != 0 && nnb[k][2] != lcn) {
        int dup = 0;
        for (l = 0; l < k; l++)
          if (nnb[l][2] == nnb[k][2]) { dup = 1; break; }
        if (!dup) {
          clsum += nnb[k][3];
          for (j = 0; j < S->nb; j++)
            if (label[j] == nnb[k][2]) label[j] = lcn;
        }
        csize[nnb[k][2]] = 0;
      }
    }
    for (j = 0; j < S->nb; j++)
      if (b1[j] == a && b2[j] == bb) label[j] = lcn;
    clsum++;
    csize[lcn] = clsum;
  }
  if (csize[lcn] > S->maxcs) {
    S->maxcs = csize[lcn];
    S->maxcn = lcn;
  } else if (lcs == 0) {
    if (S->maxcs == 0) { S->maxcs = 1; S->maxcn = 1; }
  }
}

int or_label_bonds_literal(int lattice, int m, int n, int pbc, int nb,
                           const int *b1, const int *b2,
                           const int *o1, const int *o2, int tbonds,
                           int *label, int *csize, int *maxcn_o, int *maxcs_o) {
  lit_state S;
  int i;
  S.lattice = lattice; S.m = m; S.n = n; S.pbc = pbc; S.nb = nb;
  S.scn = or_scn(lattice); S.bcn = or_bcn(lattice);
  S.b1 = b1; S.b2 = b2; S.label = label; S.csize = csize;
  S.cln = 1; S.maxcn = 0; S.maxcs = 0;
  memset(label, 0, sizeof(int) * (size_t)nb);
  memset(csize, 0, sizeof(int) * (size_t)(nb + 2));
  for (i = 1; i <= tbonds; i++) lit_add_bond(&S, o1[i - 1], o2[i - 1]);
  if (maxcn_o) *maxcn_o = S.maxcn;
  if (maxcs_o) *maxcs_o = S.maxcs;
  return S.cln;
}

/* ---- union-find helpers for the replays ------------------------------ */
static int uf_find(int *par, int x) {
  int r = x;
  while (par[r] != r) r = par[r];
  while (par[x] != r) { int nx = par[x]; par[x] = r; x = nx; }
  return r;
}
static int uf_union(int *par, int *sz, int a, int b) {
  int ra = uf_find(par, a), rb = uf_find(par, b);
  if (ra == rb) return ra;
  if (sz[ra] < sz[rb]) { int tmp = ra; ra = rb; rb = tmp; }
  par[rb] = ra;
  sz[ra] += sz[rb];
  return ra;
}

/* bond index of pair (p<q) in the bond list, -1 if not a lattice bond */
typedef struct { int *first; const int *b2; int t; } bond_index;
static int bidx(const bond_index *bi, int p, int q) {
  int k;
  if (p < 1 || p > bi->t) return -1;
  for (k = bi->first[p]; k < bi->first[p + 1]; k++)
    if (bi->b2[k] == q) return k;
  return -1;
}

/* Bond labeling, union-find replay with the literal loop's semantics.
   Returns -2 if the neighbour relation is asymmetric in a way the replay
   cannot express (triangular odd m, hazard H7): use the literal form. */
int or_label_bonds_replay(int lattice, int m, int n, int pbc, int nb,
                          const int *b1, const int *b2,
                          const int *o1, const int *o2, int tbonds,
                          int *label, int *csize, int *maxcn_o, int *maxcs_o) {
  int t = m * n, scn = or_scn(lattice);
  int i, j, k, cln = 1, maxcn = 0, maxcs = 0, nn[6], ret = 0;
  int *par = (int *)malloc(sizeof(int) * (size_t)(t + 2));
  int *sz = (int *)malloc(sizeof(int) * (size_t)(t + 2));
  int *clab = (int *)malloc(sizeof(int) * (size_t)(t + 2));
  unsigned char *occ = (unsigned char *)calloc((size_t)nb + 1, 1);
  bond_index bi;
  bi.first = (int *)calloc((size_t)t + 2, sizeof(int));
  bi.b2 = b2;
  bi.t = t;
  for (k = 0; k < nb; k++) bi.first[b1[k] + 1]++;
  for (i = 1; i <= t + 1; i++) bi.first[i] += bi.first[i - 1];
  for (i = 0; i <= t + 1; i++) { par[i] = i; sz[i] = 1; clab[i] = 0; }
  memset(csize, 0, sizeof(int) * (size_t)(nb + 2));

  for (i = 1; i <= tbonds; i++) {
    int a = o1[i - 1], bb = o2[i - 1];
    int rows[10][2], rlab[10], rsize[10], rc = 0, lcn, lcs, clsum, self, r;
    if (a <= 0) {
      /* H2 sentinel (0,0): no nnb row matches a real bond and no b row
         matches (0,0): the reference opens a phantom cluster. */
      csize[cln] = 1;
      cln++;
      if (maxcs == 0) { maxcs = 1; maxcn = 1; }
      continue;
    }
    or_nearestn(lattice, m, n, pbc, a, nn);
    for (j = 0; j < scn; j++)
      if (nn[j] != 0 && nn[j] != bb) {
        rows[rc][0] = nn[j] > a ? a : nn[j];
        rows[rc][1] = nn[j] > a ? nn[j] : a;
        rc++;
      }
    or_nearestn(lattice, m, n, pbc, bb, nn);
    for (j = 0; j < scn; j++)
      if (nn[j] != 0 && nn[j] != a) {
        rows[rc][0] = nn[j] > bb ? bb : nn[j];
        rows[rc][1] = nn[j] > bb ? nn[j] : bb;
        rc++;
      }
    for (k = 0; k < rc; k++) {
      int q = bidx(&bi, rows[k][0], rows[k][1]);
      if (q >= 0 && occ[q]) {
        rlab[k] = clab[uf_find(par, rows[k][0])];
        rsize[k] = csize[rlab[k]];
      } else {
        rlab[k] = 0;
        rsize[k] = 0;
      }
    }
    lcn = rc > 0 ? rlab[0] : 0;
    lcs = rc > 0 ? rsize[0] : 0;
    for (k = 1; k < rc; k++)
      if (rlab[k] != 0 && rsize[k] > lcs) { lcn = rlab[k]; lcs = rsize[k]; }
    self = bidx(&bi, a, bb);
    if (self < 0) { ret = -3; break; }
    if (lcs == 0) {
      if (clab[uf_find(par, a)] != 0 || clab[uf_find(par, bb)] != 0) {
        ret = -2; /* H7: a cluster at an endpoint is not among the rows */
        break;
      }
      occ[self] = 1;
      r = uf_union(par, sz, a, bb);
      clab[r] = cln;
      csize[cln] = 1;
      cln++;
    } else {
      clsum = lcs;
      for (k = 0; k < rc; k++) {
        if (rlab[k] != 0 && rlab[k] != lcn) {
          int l, dup = 0;
          for (l = 0; l < k; l++)
            if (rlab[l] == rlab[k]) { dup = 1; break; }
          if (!dup) {
            clsum += rsize[k];
            uf_union(par, sz, a, rows[k][0]);
          }
          csize[rlab[k]] = 0;
        } else if (rlab[k] == lcn && rlab[k] != 0) {
          uf_union(par, sz, a, rows[k][0]);
        }
      }
      occ[self] = 1;
      r = uf_union(par, sz, a, bb);
      clab[r] = lcn;
      clsum++;
      csize[lcn] = clsum;
    }
    if (csize[lcn] > maxcs) {
      maxcs = csize[lcn];
      maxcn = lcn;
    } else if (lcs == 0) {
      if (maxcs == 0) { maxcs = 1; maxcn = 1; }
    }
  }
  for (k = 0; k < nb; k++)
    label[k] = occ[k] ? clab[uf_find(par, b1[k])] : 0;
  free(par); free(sz); free(clab); free(occ); free(bi.first);
  if (maxcn_o) *maxcn_o = maxcn;
  if (maxcs_o) *maxcs_o = maxcs;
  return ret ? ret : cln;
}

/* ======================================================================
 * Site labeling.  Square/site.f:162-289.
 * ==================================================================== */
int or_label_sites_literal(int lattice, int m, int n, int pbc,
                           const int *order, int tsites,
                           int *s, int *csize, int *maxcn_o, int *maxcs_o) {
  int t = m * n, scn = or_scn(lattice);
  int i, j, k, l, cln = 1, maxcn = 0, maxcs = 0, nn[6], oldcn = 0;
  /* s is indexed 1..t here via sp[] (sp[0] = s(0) = 0 read for nn == 0) */
  int *sp = (int *)calloc((size_t)t + 1, sizeof(int));
  memset(csize, 0, sizeof(int) * (size_t)(t + 2));
  for (i = 1; i <= tsites; i++) {
    int sn = order[i - 1], lcn, lcs, nnlc, clsum;
    if (sn <= 0) continue; /* H2 sentinel: reference reads s(-1); skipped */
    or_nearestn(lattice, m, n, pbc, sn, nn);
    lcn = sp[nn[0]];
    lcs = csize[sp[nn[0]]];
    nnlc = nn[0];
    for (k = 1; k < scn; k++)
      if (nn[k] != 0 && sp[nn[k]] != 0 && csize[sp[nn[k]]] > lcs) {
        lcn = sp[nn[k]];
        lcs = csize[sp[nn[k]]];
        nnlc = nn[k];
      }
    if (lcs == 0) {
      sp[sn] = cln;
      csize[cln] = 1;
      cln++;
    } else {
      clsum = lcs;
      for (k = 0; k < scn; k++) {
        if (nn[k] != 0 && sp[nn[k]] != 0 && sp[nn[k]] != sp[nnlc]) {
          int dup = 0;
          for (l = 0; l < k; l++)
            if (sp[nn[l]] == sp[nn[k]]) { dup = 1; break; }
          if (!dup) {
            clsum += csize[sp[nn[k]]];
            oldcn = sp[nn[k]];
            for (j = 1; j <= t; j++)
              if (sp[j] == oldcn) sp[j] = lcn;
          }
          csize[oldcn] = 0;
        }
      }
      sp[sn] = lcn;
      clsum++;
      csize[lcn] = clsum;
    }
    if (csize[lcn] > maxcs) {
      maxcs = csize[lcn];
      maxcn = lcn;
    } else if (lcs == 0) {
      if (maxcs == 0) { maxcs = 1; maxcn = 1; }
    }
  }
  for (j = 1; j <= t; j++) s[j - 1] = sp[j];
  free(sp);
  if (maxcn_o) *maxcn_o = maxcn;
  if (maxcs_o) *maxcs_o = maxcs;
  return cln;
}

int or_label_sites_replay(int lattice, int m, int n, int pbc,
                          const int *order, int tsites,
                          int *s, int *csize, int *maxcn_o, int *maxcs_o) {
  int t = m * n, scn = or_scn(lattice);
  int i, k, cln = 1, maxcn = 0, maxcs = 0, nn[6];
  int *par = (int *)malloc(sizeof(int) * (size_t)(t + 1));
  int *sz = (int *)malloc(sizeof(int) * (size_t)(t + 1));
  int *clab = (int *)calloc((size_t)t + 1, sizeof(int));
  unsigned char *occ = (unsigned char *)calloc((size_t)t + 1, 1);
  for (i = 0; i <= t; i++) { par[i] = i; sz[i] = 1; }
  memset(csize, 0, sizeof(int) * (size_t)(t + 2));
  for (i = 1; i <= tsites; i++) {
    int sn = order[i - 1], lab[6] = {0}, siz[6] = {0}, lcn, lcs, clsum, r;
    if (sn <= 0) continue;
    or_nearestn(lattice, m, n, pbc, sn, nn);
    for (k = 0; k < scn; k++) {
      if (nn[k] > 0 && occ[nn[k]]) {
        lab[k] = clab[uf_find(par, nn[k])];
        siz[k] = csize[lab[k]];
      } else {
        lab[k] = 0;
        siz[k] = 0;
      }
    }
    lcn = lab[0];
    lcs = siz[0];
    for (k = 1; k < scn; k++)
      if (nn[k] != 0 && lab[k] != 0 && siz[k] > lcs) { lcn = lab[k]; lcs = siz[k]; }
    occ[sn] = 1;
    if (lcs == 0) {
      clab[sn] = cln;
      csize[cln] = 1;
      cln++;
    } else {
      clsum = lcs;
      for (k = 0; k < scn; k++) {
        if (nn[k] != 0 && lab[k] != 0) {
          int l, dup = 0;
          if (lab[k] != lcn) {
            for (l = 0; l < k; l++)
              if (lab[l] == lab[k]) { dup = 1; break; }
            if (!dup) {
              clsum += siz[k];
              csize[lab[k]] = 0;
            }
          }
          uf_union(par, sz, sn, nn[k]);
        }
      }
      r = uf_find(par, sn);
      clab[r] = lcn;
      clsum++;
      csize[lcn] = clsum;
    }
    if (csize[lcn] > maxcs) {
      maxcs = csize[lcn];
      maxcn = lcn;
    } else if (lcs == 0) {
      if (maxcs == 0) { maxcs = 1; maxcn = 1; }
    }
  }
  for (i = 1; i <= t; i++) s[i - 1] = occ[i] ? clab[uf_find(par, i)] : 0;
  free(par); free(sz); free(clab); free(occ);
  if (maxcn_o) *maxcn_o = maxcn;
  if (maxcs_o) *maxcs_o = maxcs;
  return cln;
}

/* ======================================================================
 * Mixed site-then-bond labeling, literal.  Square/sitebond.f:187-400.
 * ==================================================================== */
int or_label_sitebond(int lattice, int m, int n, int pbc, int nb,
                      const int *b1, const int *b2,
                      const int *sorder, int tsites,
                      const int *o1, const int *o2, int tbonds,
                      int *s, int *blabel, int *csize, int *maxcn_o,
                      int *maxcs_o) {
  int t = m * n, i, j, k, cln = 1, maxcn, maxcs, lcn = 0, lcs = 0;
  int *sp = (int *)calloc((size_t)t + 1, sizeof(int));
  (void)lattice; (void)pbc;
  memset(blabel, 0, sizeof(int) * (size_t)nb);
  memset(csize, 0, sizeof(int) * (size_t)(t + nb + 2));
  for (i = 1; i <= tsites; i++) { /* sitebond.f:187-196 */
    int sn = sorder[i - 1];
    if (sn > 0) sp[sn] = cln;
    csize[cln] = 1;
    cln++;
  }
  maxcn = 1;
  maxcs = 1;
  for (i = 1; i <= tbonds; i++) { /* sitebond.f:223-400 */
    for (j = 0; j < nb; j++) {
      if (b1[j] == o1[i - 1] && b2[j] == o2[i - 1]) {
        int sa = sp[b1[j]], sb = sp[b2[j]], oldcn, clsum;
        if (sa == 0 && sb == 0) {
          blabel[j] = cln; csize[cln] = 1; cln++;
          break;
        }
        if (sa > 0 && sb == 0) {
          lcn = sa; lcs = csize[sa]; blabel[j] = lcn; csize[sa] = lcs + 1;
          break;
        }
        if (sa == 0 && sb > 0) {
          lcn = sb; lcs = csize[sb]; blabel[j] = lcn; csize[sb] = lcs + 1;
          break;
        }
        if (sa == sb) {
          lcn = sa; lcs = csize[sa]; blabel[j] = lcn; csize[sa] = lcs + 1;
          break;
        }
        if (csize[sa] > csize[sb]) { lcn = sa; oldcn = sb; }
        else { lcn = sb; oldcn = sa; }
        lcs = csize[lcn];
        blabel[j] = lcn;
        clsum = lcs + csize[oldcn] + 1;
        for (k = 1; k <= t; k++)
          if (sp[k] == oldcn) sp[k] = lcn;
        for (k = 0; k < nb; k++)
          if (blabel[k] == oldcn) blabel[k] = lcn;
        csize[oldcn] = 0;
        csize[lcn] = clsum;
        break;
      }
    }
    if (csize[lcn] > maxcs) { maxcs = csize[lcn]; maxcn = lcn; }
  }
  for (j = 1; j <= t; j++) s[j - 1] = sp[j];
  free(sp);
  if (maxcn_o) *maxcn_o = maxcn;
  if (maxcs_o) *maxcs_o = maxcs;
  return cln;
}

/* Mixed site-then-bond labeling, union-find replay of or_label_sitebond
   (Square/sitebond.f:187-400): the same labels, sizes, cln and maxcn/maxcs,
   in O(N alpha).  A merge relabels oldcn -> lcn everywhere
   (sitebond.f:330-352); here label oldcn is linked to lcn in a union-find
   over label ids and every stored label is resolved through it. */
static int lab_find(int *lp, int x) {
  int r = x;
  while (lp[r] != r) r = lp[r];
  while (lp[x] != r) { int nx = lp[x]; lp[x] = r; x = nx; }
  return r;
}
int or_label_sitebond_replay(int lattice, int m, int n, int pbc, int nb,
                             const int *b1, const int *b2,
                             const int *sorder, int tsites,
                             const int *o1, const int *o2, int tbonds,
                             int *s, int *blabel, int *csize, int *maxcn_o,
                             int *maxcs_o) {
  int t = m * n, i, j, k, cln = 1, maxcn, maxcs, lcn = 0, lcs = 0;
  size_t cap = (size_t)t + (size_t)nb + 2;
  int *sp = (int *)calloc((size_t)t + 1, sizeof(int));
  int *lp = (int *)malloc(sizeof(int) * cap);
  bond_index bi;
  (void)lattice; (void)pbc;
  bi.first = (int *)calloc((size_t)t + 2, sizeof(int));
  bi.b2 = b2;
  bi.t = t;
  for (k = 0; k < nb; k++) bi.first[b1[k] + 1]++;
  for (i = 1; i <= t + 1; i++) bi.first[i] += bi.first[i - 1];
  for (k = 0; k < (int)cap; k++) lp[k] = k;
  memset(blabel, 0, sizeof(int) * (size_t)nb);
  memset(csize, 0, sizeof(int) * cap);
  for (i = 1; i <= tsites; i++) { /* sitebond.f:187-196 */
    int sn = sorder[i - 1];
    if (sn > 0) sp[sn] = cln;
    csize[cln] = 1;
    cln++;
  }
  maxcn = 1;
  maxcs = 1;
  for (i = 1; i <= tbonds; i++) { /* sitebond.f:223-400 */
    int a = o1[i - 1], bb = o2[i - 1];
    j = a > 0 ? bidx(&bi, a, bb) : -1; /* the (0,0) spill matches no bond */
    if (j >= 0) {
      int sa = sp[b1[j]] ? lab_find(lp, sp[b1[j]]) : 0;
      int sb = sp[b2[j]] ? lab_find(lp, sp[b2[j]]) : 0, oldcn;
      if (sa == 0 && sb == 0) {
        blabel[j] = cln; csize[cln] = 1; cln++;
      } else if (sa > 0 && sb == 0) {
        lcn = sa; lcs = csize[sa]; blabel[j] = lcn; csize[sa] = lcs + 1;
      } else if (sa == 0 && sb > 0) {
        lcn = sb; lcs = csize[sb]; blabel[j] = lcn; csize[sb] = lcs + 1;
      } else if (sa == sb) {
        lcn = sa; lcs = csize[sa]; blabel[j] = lcn; csize[sa] = lcs + 1;
      } else {
        if (csize[sa] > csize[sb]) { lcn = sa; oldcn = sb; }
        else { lcn = sb; oldcn = sa; }
        lcs = csize[lcn];
        blabel[j] = lcn;
        lp[oldcn] = lcn;
        csize[lcn] = lcs + csize[oldcn] + 1;
        csize[oldcn] = 0;
      }
    }
    if (csize[lcn] > maxcs) { maxcs = csize[lcn]; maxcn = lcn; }
  }
  for (j = 1; j <= t; j++) s[j - 1] = sp[j] ? lab_find(lp, sp[j]) : 0;
  for (j = 0; j < nb; j++) blabel[j] = blabel[j] ? lab_find(lp, blabel[j]) : 0;
  free(sp);
  free(lp);
  free(bi.first);
  if (maxcn_o) *maxcn_o = maxcn;
  if (maxcs_o) *maxcs_o = maxcs;
  return cln;
}

/* Canonical partition ids (test helpers): canon[s-1] = the minimum site of
   the cluster site s belongs to, 0 for a site in no cluster.  Sites: by the
   site label s[]; bonds: a site is in the cluster of every occupied bond
   (label > 0) it ends. */
void or_canon_sites(int t, const int *s, int maxlab, int *canon) {
  int *mins = (int *)malloc(sizeof(int) * ((size_t)maxlab + 1)), k;
  for (k = 0; k <= maxlab; k++) mins[k] = 0;
  for (k = 1; k <= t; k++) {
    int l = s[k - 1];
    if (l > 0 && mins[l] == 0) mins[l] = k; /* ascending k: first = min */
  }
  for (k = 1; k <= t; k++) canon[k - 1] = s[k - 1] > 0 ? mins[s[k - 1]] : 0;
  free(mins);
}
void or_canon_bonds(int t, int nb, const int *b1, const int *b2, const int *label, int maxlab,
                    int *canon) {
  int *mins = (int *)malloc(sizeof(int) * ((size_t)maxlab + 1)), k;
  for (k = 0; k <= maxlab; k++) mins[k] = 0;
  for (k = 0; k < nb; k++) {
    int l = label[k];
    if (l > 0 && (mins[l] == 0 || b1[k] < mins[l])) mins[l] = b1[k];
  }
  for (k = 0; k < t; k++) canon[k] = 0;
  for (k = 0; k < nb; k++)
    if (label[k] > 0) canon[b1[k] - 1] = canon[b2[k] - 1] = mins[label[k]];
  free(mins);
}

/* ======================================================================
 * Mixed bonds-then-sites labeling, literal.  Square/bondsite.f:170-322
 * (Triangular/bondsite.f: the same loops, scn 6).  border = shuffled bond
 * ids (0 = the shuffle's spill slot), sorder = shuffled sites.  s[t],
 * blabel[nb], csize[cap >= t + nb + 2] (c(0) = csize[0] stays 0: the
 * reference reads c(0) for an unoccupied first neighbour bond, and in its
 * build that word is 0).  Returns cln.
 * ==================================================================== */
int or_label_bondsite(int lattice, int m, int n, int pbc, int nb,
                      const int *b1, const int *b2,
                      const int *border, int tbonds,
                      const int *sorder, int tsites,
                      int *s, int *blabel, int *csize, int *maxcn_o,
                      int *maxcs_o) {
  int t = m * n, i, j, k, l, cln = 1, maxcn = 1, maxcs = 1;
  int *sp = (int *)calloc((size_t)t + 1, sizeof(int));
  memset(blabel, 0, sizeof(int) * (size_t)nb);
  memset(csize, 0, sizeof(int) * (size_t)(t + nb + 2));
  for (i = 1; i <= tbonds; i++) { /* bondsite.f:182-199 */
    int id = border[i - 1];
    if (id > 0) blabel[id - 1] = cln; /* b(j,3) = cln for the matching row */
    csize[cln] = 1;
    cln++;
  }
  for (i = 1; i <= tsites; i++) { /* bondsite.f:220-320 */
    int sn = sorder[i - 1], nn[10], nnb[12][4], rc = 0, lcn, lcs, clsum;
    memset(nnb, 0, sizeof(nnb));
    if (sn <= 0) { /* spill slot: no neighbour bond matches -> case 1 */
      csize[cln] = 1;
      cln++;
      lcn = 0;
      goto track;
    }
    or_nearestn(lattice, m, n, pbc, sn, nn);
    for (j = 0; j < (lattice ? 6 : 4); j++) {
      if (nn[j] != 0) {
        nnb[rc][0] = nn[j] > sn ? sn : nn[j];
        nnb[rc][1] = nn[j] > sn ? nn[j] : sn;
        rc++;
      }
    }
    for (j = 0; j < nb; j++) /* bondsite.f:245-254 */
      for (k = 0; k < (lattice ? 6 : 4); k++)
        if (b1[j] == nnb[k][0] && b2[j] == nnb[k][1]) {
          nnb[k][2] = blabel[j];
          nnb[k][3] = csize[blabel[j]];
        }
    lcn = nnb[0][2];
    lcs = nnb[0][3];
    for (k = 1; k < (lattice ? 6 : 4); k++) /* bondsite.f:262-272 */
      if (nnb[k][0] != 0 && nnb[k][2] != 0 && nnb[k][3] > lcs) {
        lcn = nnb[k][2];
        lcs = nnb[k][3];
      }
    if (lcs == 0) { /* case 1 */
      sp[sn] = cln;
      csize[cln] = 1;
      cln++;
      goto track;
    }
    clsum = lcs; /* case 2 */
    for (k = 0; k < (lattice ? 6 : 4); k++) {
      if (nnb[k][0] == 0 || nnb[k][2] == 0 || nnb[k][2] == lcn) continue;
      {
        int dup = 0;
        for (l = 0; l < k; l++) if (nnb[l][2] == nnb[k][2]) dup = 1;
        if (!dup) {
          clsum += nnb[k][3];
          for (j = 0; j < nb; j++) if (blabel[j] == nnb[k][2]) blabel[j] = lcn;
          for (j = 1; j <= t; j++) if (sp[j] == nnb[k][2]) sp[j] = lcn;
        }
      }
      csize[nnb[k][2]] = 0;
    }
    sp[sn] = lcn;
    clsum = clsum + 1;
    csize[lcn] = clsum;
  track:
    if (csize[lcn] > maxcs) { maxcs = csize[lcn]; maxcn = lcn; }
  }
  for (j = 1; j <= t; j++) s[j - 1] = sp[j];
  free(sp);
  if (maxcn_o) *maxcn_o = maxcn;
  if (maxcs_o) *maxcs_o = maxcs;
  return cln;
}

/* ======================================================================
 * Spanning detection.
 * ==================================================================== */
int or_span_bonds(int m, int n, int nb, const int *b1, const int *b2,
                  const int *label, const int *csize, int cln) {
  /* Square/bondc.f:413-456: first (lowest) label wins */
  int t = m * n, l, k;
  unsigned char *bot = (unsigned char *)calloc((size_t)cln + 1, 1);
  unsigned char *top = (unsigned char *)calloc((size_t)cln + 1, 1);
  int res = 0;
  for (k = 0; k < nb; k++) {
    int lab = label[k];
    if (lab <= 0 || lab >= cln) continue;
    if (b1[k] >= 1 && b1[k] <= m) bot[lab] = 1;
    if (b2[k] > t - m && b2[k] <= t) top[lab] = 1;
  }
  for (l = 1; l < cln; l++)
    if (csize[l] >= n - 1 && bot[l] && top[l]) { res = l; break; }
  free(bot); free(top);
  return res;
}

int or_span_sites(int m, int n, const int *s, const int *csize, int cln,
                  int minsize) {
  /* Square/site.f:309-344 (minsize n), Square/sitebond.f:423-458 (2n-1) */
  int t = m * n, l, j, res = 0;
  unsigned char *bot = (unsigned char *)calloc((size_t)cln + 1, 1);
  unsigned char *top = (unsigned char *)calloc((size_t)cln + 1, 1);
  (void)n;
  for (j = 1; j <= m; j++) if (s[j - 1] > 0 && s[j - 1] < cln) bot[s[j - 1]] = 1;
  for (j = t - m + 1; j <= t; j++)
    if (s[j - 1] > 0 && s[j - 1] < cln) top[s[j - 1]] = 1;
  for (l = 1; l < cln; l++)
    if (csize[l] >= minsize && bot[l] && top[l]) { res = l; break; }
  free(bot); free(top);
  return res;
}

/* ======================================================================
 * Conductance.
 * ==================================================================== */
void or_bond_values(int rule, int nb, const int *b1, const int *b2,
                    const int *blabel, const int *s, int perccln, double g0,
                    double leak, double *gval) {
  int k;
  for (k = 0; k < nb; k++) {
    int in;
    if (rule == 0) /* Square/bondc.f:483-489 */
      in = blabel[k] == perccln;
    else if (rule == 1) /* MATLAB/ConductCalc.m:90 */
      in = s[b1[k] - 1] == perccln && s[b2[k] - 1] == perccln;
    else /* MATLAB/ConductCalc.m:136-137 */
      in = blabel[k] == perccln && s[b1[k] - 1] == perccln &&
           s[b2[k] - 1] == perccln;
    gval[k] = in ? -g0 : -leak;
  }
}

/* per-site adjacency sorted by column (dense-row scan order of G) */
typedef struct { int *start; int *col; double *val; } adj_t;

static void build_adj(int t, int nb, const int *b1, const int *b2,
                      const double *gval, adj_t *A) {
  int k, i;
  int *cnt = (int *)calloc((size_t)t + 2, sizeof(int));
  A->start = (int *)calloc((size_t)t + 2, sizeof(int));
  A->col = (int *)malloc(sizeof(int) * (size_t)(2 * nb + 1));
  A->val = (double *)malloc(sizeof(double) * (size_t)(2 * nb + 1));
  for (k = 0; k < nb; k++) { A->start[b1[k] + 1]++; A->start[b2[k] + 1]++; }
  for (i = 1; i <= t + 1; i++) A->start[i] += A->start[i - 1];
  for (k = 0; k < nb; k++) {
    int p = b1[k], q = b2[k];
    A->col[A->start[p] + cnt[p]] = q; A->val[A->start[p] + cnt[p]] = gval[k]; cnt[p]++;
    A->col[A->start[q] + cnt[q]] = p; A->val[A->start[q] + cnt[q]] = gval[k]; cnt[q]++;
  }
  /* insertion sort each row by column (<= 6 entries) */
  for (i = 1; i <= t; i++) {
    int a = A->start[i], e = A->start[i + 1], x, y;
    for (x = a + 1; x < e; x++) {
      int c = A->col[x]; double v = A->val[x];
      y = x - 1;
      while (y >= a && A->col[y] > c) {
        A->col[y + 1] = A->col[y]; A->val[y + 1] = A->val[y]; y--;
      }
      A->col[y + 1] = c; A->val[y + 1] = v;
    }
  }
  free(cnt);
}
static void free_adj(adj_t *A) { free(A->start); free(A->col); free(A->val); }

int or_assemble(int lattice, int m, int n, int pbc, int nb, const int *b1,
                const int *b2, const double *gval, double Va, double thresh,
                int rhs_rule, int nmax, double *sa, int *ija, double *itemp,
                double *diag_full) {
  int t = m * n, N = t - 2 * m, i, k, x;
  adj_t A;
  (void)lattice; (void)pbc;
  build_adj(t, nb, b1, b2, gval, &A);
  /* diagonal: G(i,i) = -sum_j G(i,j), ascending j (Square/bondc.f:499-505) */
  for (i = 1; i <= t; i++) {
    double rowsum = 0.0;
    for (x = A.start[i]; x < A.start[i + 1]; x++) rowsum = rowsum + A.val[x];
    diag_full[i - 1] = -rowsum;
  }
  /* RHS (Square/bondc.f:490-497; MATLAB/ConductCalc.m:126-130) */
  for (i = 0; i < N; i++) itemp[i] = 0.0;
  for (k = 0; k < nb; k++) {
    if (b1[k] > t - 2 * m && b1[k] <= t - m && b2[k] > t - m) {
      int r = b1[k] - m - 1;
      if (rhs_rule == 0) itemp[r] = itemp[r] - (gval[k] * Va);
      else itemp[r] = itemp[r] + (-gval[k] * Va);
    }
  }
  /* sprsin on Gtemp = G(m+1..t-m, m+1..t-m) (Square/bondc.f:723-746) */
  if (N + 1 > nmax) { free_adj(&A); return -1; }
  for (i = 1; i <= N; i++) sa[i - 1] = diag_full[i + m - 1];
  ija[0] = N + 2;
  k = N + 1;
  for (i = 1; i <= N; i++) {
    int site = i + m;
    for (x = A.start[site]; x < A.start[site + 1]; x++) {
      int c = A.col[x];
      if (c <= m || c > t - m) continue;
      if (fabs(A.val[x]) >= thresh) {
        k++;
        if (k > nmax) { free_adj(&A); return -1; }
        sa[k - 1] = A.val[x];
        ija[k - 1] = c - m;
      }
    }
    ija[i] = k + 1;
  }
  free_adj(&A);
  return k;
}

void or_dsprsax(const double *sa, const int *ija, const double *x, double *b,
                int n) {
  /* Square/bondc.f:887-899 */
  int i, k;
  for (i = 1; i <= n; i++) {
    double acc = sa[i - 1] * x[i - 1];
    for (k = ija[i - 1]; k <= ija[i] - 1; k++)
      acc = acc + sa[k - 1] * x[ija[k - 1] - 1];
    b[i - 1] = acc;
  }
}

void or_dsprstx(const double *sa, const int *ija, const double *x, double *b,
                int n) {
  /* Square/bondc.f:902-917 */
  int i, k;
  for (i = 1; i <= n; i++) b[i - 1] = sa[i - 1] * x[i - 1];
  for (i = 1; i <= n; i++)
    for (k = ija[i - 1]; k <= ija[i] - 1; k++) {
      int j = ija[k - 1];
      b[j - 1] = b[j - 1] + sa[k - 1] * x[i - 1];
    }
}

static double snrm2(int n, const double *sx) {
  /* Square/bondc.f:867-884, itol <= 3 */
  double s = 0.0;
  int i;
  for (i = 0; i < n; i++) s = s + sx[i] * sx[i];
  return sqrt(s);
}

static double snrm_itol(int n, const double *sx, int itol) {
  /* Square/bondc.f:867-884: sum of squares for itol <= 3, else the first
     largest |sx(i)| */
  int i, im = 0;
  if (itol <= 3) return snrm2(n, sx);
  for (i = 1; i < n; i++)
    if (fabs(sx[i]) > fabs(sx[im])) im = i;
  return fabs(sx[im]);
}

void or_linbcg(const double *sa, const int *ija, int n, const double *b,
               double *x, int itol, double tol, int itmax, int *iter_o,
               double *err_o, double *iter_err) {
  /* Square/bondc.f:750-838, literal (itol 1..4) */
  double *p = (double *)calloc((size_t)n, sizeof(double));
  double *pp = (double *)calloc((size_t)n, sizeof(double));
  double *r = (double *)calloc((size_t)n, sizeof(double));
  double *rr = (double *)calloc((size_t)n, sizeof(double));
  double *z = (double *)calloc((size_t)n, sizeof(double));
  double *zz = (double *)calloc((size_t)n, sizeof(double));
  const double EPS = 1.00e-14; /* bondc.f:753 */
  double ak, akden, bk, bkden = 1.0, bknum, bnrm, err = 0.0, znrm = 1.0, zm1nrm;
  int j, iter = 0;
  or_dsprsax(sa, ija, x, r, n);
  for (j = 0; j < n; j++) { r[j] = b[j] - r[j]; rr[j] = r[j]; }
  if (itol == 1) {
    bnrm = snrm2(n, b);
  } else {
    for (j = 0; j < n; j++) z[j] = b[j] / sa[j];
    bnrm = snrm_itol(n, z, itol);
    if (itol >= 3) { /* bondc.f:771-775 */
      for (j = 0; j < n; j++) z[j] = r[j] / sa[j];
      znrm = snrm_itol(n, z, itol);
    }
  }
  for (j = 0; j < n; j++) z[j] = r[j] / sa[j];
  while (iter <= itmax) {
    iter++;
    zm1nrm = znrm;
    for (j = 0; j < n; j++) zz[j] = rr[j] / sa[j];
    bknum = 0.0;
    for (j = 0; j < n; j++) bknum = bknum + z[j] * rr[j];
    if (iter == 1) {
      for (j = 0; j < n; j++) { p[j] = z[j]; pp[j] = zz[j]; }
    } else {
      bk = bknum / bkden;
      for (j = 0; j < n; j++) {
        p[j] = bk * p[j] + z[j];
        pp[j] = bk * pp[j] + zz[j];
      }
    }
    bkden = bknum;
    or_dsprsax(sa, ija, p, z, n);
    akden = 0.0;
    for (j = 0; j < n; j++) akden = akden + z[j] * pp[j];
    ak = bknum / akden;
    or_dsprstx(sa, ija, pp, zz, n);
    for (j = 0; j < n; j++) {
      x[j] = x[j] + ak * p[j];
      r[j] = r[j] - ak * z[j];
      rr[j] = rr[j] - ak * zz[j];
    }
    for (j = 0; j < n; j++) z[j] = r[j] / sa[j];
    if (itol <= 2) {
      err = snrm2(n, r) / bnrm;
    } else { /* bondc.f:816-832: the step-size estimate; the goto 100
                branches iterate on without the tolerance test */
      znrm = snrm_itol(n, z, itol);
      if (iter_err) iter_err[iter - 1] = znrm / bnrm;
      if (fabs(zm1nrm - znrm) > EPS * znrm) {
        err = znrm / fabs(zm1nrm - znrm) * (fabs(ak) * snrm_itol(n, p, itol));
      } else {
        err = znrm / bnrm;
        continue;
      }
      {
        const double xnrm = snrm_itol(n, x, itol);
        if (err <= 0.50 * xnrm) {
          err = err / xnrm;
        } else {
          err = znrm / bnrm;
          continue;
        }
      }
    }
    if (iter_err) iter_err[iter - 1] = err;
    if (!(err > tol)) break;
  }
  *iter_o = iter;
  *err_o = err;
  free(p); free(pp); free(r); free(rr); free(z); free(zz);
}

/* The same linbcg (itol 2), for fixtures at the BASELINE config sizes:
   bitwise the literal or_linbcg's iterates on a bitwise-symmetric matrix,
   several times faster, with snapshots of x at a list of tolerances from one
   run.  Why it is the same arithmetic (Square/bondc.f:750-838):
   * for a bitwise-symmetric sa, dsprstx (bondc.f:902-917) forms every b(j)
     as diagonal first, then the rows i of column j in ascending order --
     which are row j's columns in ascending order with the same values, i.e.
     exactly dsprsax's sum.  So rr == r, pp == p, zz == z
     bit for bit and one copy of each suffices;
   * every per-element update and every SpMV row is computed as in or_linbcg,
     only split over threads (no element's operation order changes);
   * the three dot products stay serial sums in ascending j (the literal
     association); ||r||^2 and the next iteration's z.r (both over the same
     r) run as two serial chains side by side.
   Snapshot c is x at the first iteration with !(err > check_tols[c])
   (check_tols descending) -- the x a literal run with tol = check_tols[c]
   returns.  Returns 0, or -1 (nothing computed) if sa is not bitwise
   symmetric. */
static int sym_entry(const double *sa, const int *ija, int row, int col,
                     double *v) {
  int k;
  for (k = ija[row - 1]; k <= ija[row] - 1; k++)
    if (ija[k - 1] == col) { *v = sa[k - 1]; return 1; }
  return 0;
}
/* dot_order 1 (not the reference's): the same solver with its three dot
   products summed in descending j instead -- one other association, to
   measure how far the converged Gtop / Gbot of the reference solver itself
   move when only the order of its sums changes. */
/* dot_order 2: pairwise (tree) summation, halving down to runs of 8 summed
   serially -- the association family of a GPU reduction (wave and
   workgroup trees), with far smaller rounding growth than a serial sum */
static double dot_tree(int n, const double *u, const double *v) {
  double s = 0.0;
  int i, h;
  if (n <= 8) {
    for (i = 0; i < n; i++) s = s + u[i] * v[i];
    return s;
  }
  h = n / 2;
  return dot_tree(h, u, v) + dot_tree(n - h, u + h, v + h);
}
/* dot_order 3: 4096 contiguous blocks, each summed serially, then the block
   sums serially -- the shape of a per-thread / per-workgroup partial sum */
static double dot_block(int n, const double *u, const double *v) {
  const int nblk = 4096;
  double s = 0.0;
  int b;
  for (b = 0; b < nblk; b++) {
    const long long i0 = (long long)n * b / nblk, i1 = (long long)n * (b + 1) / nblk;
    double t = 0.0;
    long long i;
    for (i = i0; i < i1; i++) t = t + u[i] * v[i];
    s = s + t;
  }
  return s;
}
static double dot_ord(int n, const double *u, const double *v, int desc) {
  double s = 0.0;
  int i;
  if (desc == 2) return dot_tree(n, u, v);
  if (desc == 3) return dot_block(n, u, v);
  if (desc)
    for (i = n - 1; i >= 0; i--) s = s + u[i] * v[i];
  else
    for (i = 0; i < n; i++) s = s + u[i] * v[i];
  return s;
}
int or_linbcg_sym(const double *sa, const int *ija, int n, const double *b,
                  double *x, int itmax, int nthreads, int ncheck,
                  const double *check_tols, double *check_x, int *check_iter,
                  double *check_err, int *iter_o, double *err_o,
                  double *iter_err, int dot_order) {
  double *p, *r, *z, *q;
  double ak, akden, bk, bkden = 1.0, bknum = 0.0, bnrm, err = 0.0, rr2 = 0.0;
  int j, iter = 0, c = 0, bad = 0;
  double tol = ncheck > 0 ? check_tols[ncheck - 1] : 0.0;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(static) num_threads(nthreads) reduction(|| : bad)
  for (j = 1; j <= n; j++) {
    int k;
    for (k = ija[j - 1]; k <= ija[j] - 1; k++) {
      double v;
      if (!sym_entry(sa, ija, ija[k - 1], j, &v) || v != sa[k - 1] ||
          (v == 0.0 && signbit(v) != signbit(sa[k - 1])))
        bad = 1;
    }
  }
  if (bad) return -1;
  p = (double *)calloc((size_t)n, sizeof(double));
  r = (double *)calloc((size_t)n, sizeof(double));
  z = (double *)calloc((size_t)n, sizeof(double));
  q = (double *)calloc((size_t)n, sizeof(double));
  or_dsprsax(sa, ija, x, r, n); /* once, serial: bondc.f:759 */
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (j = 0; j < n; j++) { r[j] = b[j] - r[j]; z[j] = b[j] / sa[j]; }
  bnrm = snrm2(n, z); /* itol 2: bondc.f:768-770 */
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (j = 0; j < n; j++) z[j] = r[j] / sa[j];
  bknum = dot_ord(n, z, r, dot_order);
  while (iter <= itmax) {
    iter++;
    /* bknum = z.rr was formed at the end of the previous iteration */
    if (iter == 1) {
#pragma omp parallel for schedule(static) num_threads(nthreads)
      for (j = 0; j < n; j++) p[j] = z[j];
    } else {
      bk = bknum / bkden;
#pragma omp parallel for schedule(static) num_threads(nthreads)
      for (j = 0; j < n; j++) p[j] = bk * p[j] + z[j];
    }
    bkden = bknum;
#pragma omp parallel for schedule(dynamic, 4096) num_threads(nthreads)
    for (j = 1; j <= n; j++) { /* dsprsax row j, bondc.f:887-899 */
      int k;
      double acc = sa[j - 1] * p[j - 1];
      for (k = ija[j - 1]; k <= ija[j] - 1; k++)
        acc = acc + sa[k - 1] * p[ija[k - 1] - 1];
      q[j - 1] = acc;
    }
    akden = dot_ord(n, q, p, dot_order);
    ak = bknum / akden;
#pragma omp parallel for schedule(static) num_threads(nthreads)
    for (j = 0; j < n; j++) {
      x[j] = x[j] + ak * p[j];
      r[j] = r[j] - ak * q[j];
      z[j] = r[j] / sa[j];
    }
    /* ||r||^2 (snrm, bondc.f:867-884) and the next iteration's z.rr: two
       serial chains over the same r, each in ascending j */
#pragma omp parallel sections num_threads(nthreads > 1 ? 2 : 1)
    {
#pragma omp section
      rr2 = dot_ord(n, r, r, dot_order);
#pragma omp section
      bknum = dot_ord(n, z, r, dot_order);
    }
    err = sqrt(rr2) / bnrm;
    if (iter_err) iter_err[iter - 1] = err;
    while (c < ncheck && !(err > check_tols[c])) {
      memcpy(check_x + (size_t)c * (size_t)n, x, sizeof(double) * (size_t)n);
      check_iter[c] = iter;
      check_err[c] = err;
      c++;
    }
    if (!(err > tol)) break;
  }
  *iter_o = iter;
  *err_o = err;
  free(p); free(r); free(z); free(q);
  return 0;
}

void or_currents(int lattice, int m, int n, int pbc, int nb, const int *b1,
                 const int *b2, const double *gval, const double *diag_full,
                 const double *vint, double Va, double thresh, int cur_rule,
                 double *gtop, double *gbot) {
  /* Square/bondc.f:554-592 (cur_rule 0); MATLAB/ConductCalc.m:178-196 (1) */
  int t = m * n, i, x;
  double Ibot = 0.0, Itop = 0.0, *V, *Iout;
  adj_t A;
  (void)lattice; (void)pbc;
  build_adj(t, nb, b1, b2, gval, &A);
  V = (double *)malloc(sizeof(double) * (size_t)t);
  Iout = (double *)calloc((size_t)t, sizeof(double));
  for (i = 1; i <= t; i++) {
    if (i <= m) V[i - 1] = 0.0;
    else if (i > t - m) V[i - 1] = Va;
    else V[i - 1] = vint[i - m - 1];
  }
  for (i = 1; i <= t; i++) {
    double acc;
    if (i > m && i <= t - m) continue;
    if (cur_rule == 0) {
      /* dsprsax on sprsin(G, thresh): diagonal first, then kept columns */
      acc = diag_full[i - 1] * V[i - 1];
      for (x = A.start[i]; x < A.start[i + 1]; x++)
        if (fabs(A.val[x]) >= thresh) acc = acc + A.val[x] * V[A.col[x] - 1];
    } else {
      /* dense row times V, ascending column, diagonal in place */
      int diag_done = 0;
      acc = 0.0;
      for (x = A.start[i]; x < A.start[i + 1]; x++) {
        if (!diag_done && A.col[x] > i) {
          acc = acc + diag_full[i - 1] * V[i - 1];
          diag_done = 1;
        }
        acc = acc + A.val[x] * V[A.col[x] - 1];
      }
      if (!diag_done) acc = acc + diag_full[i - 1] * V[i - 1];
    }
    Iout[i - 1] = acc;
  }
  if (cur_rule == 0) {
    for (i = 1; i <= m; i++) {
      Ibot = Ibot + Iout[i - 1];
      Itop = Itop + Iout[i + t - m - 1];
    }
  } else {
    for (i = 1; i <= m; i++) {
      Ibot = Iout[i - 1] + Ibot;
      Itop = Iout[t - i] + Itop;
    }
  }
  *gtop = Itop / Va;
  *gbot = fabs(Ibot) / Va;
  free(V); free(Iout); free_adj(&A);
}

/* ======================================================================
 * One bondc realisation (Square/bondc.f:43-608 without the text output).
 * ==================================================================== */
int or_bondc(int lattice, int m, int n, int pbc, double pb, int seed,
             double Va, double g0, int itmax, double tol, int literal,
             int *label_out, int *csize_out, int *o1_out, int *o2_out,
             or_bondc_result *res) {
  int t = m * n, nb = or_nbonds(lattice, m, n, pbc), N = t - 2 * m;
  int *b1 = (int *)malloc(sizeof(int) * (size_t)nb);
  int *b2 = (int *)malloc(sizeof(int) * (size_t)nb);
  int *o1 = (int *)calloc((size_t)nb + 1, sizeof(int));
  int *o2 = (int *)calloc((size_t)nb + 1, sizeof(int));
  int *label = label_out ? label_out : (int *)malloc(sizeof(int) * (size_t)nb);
  int *csize = csize_out ? csize_out : (int *)malloc(sizeof(int) * (size_t)(nb + 2));
  int cnt, cln, tbonds;
  memset(res, 0, sizeof(*res));
  cnt = or_bond_list(lattice, m, n, pbc, b1, b2);
  if (cnt != nb) { res->nb = cnt; return -1; }
  memcpy(o1, b1, sizeof(int) * (size_t)nb);
  memcpy(o2, b2, sizeof(int) * (size_t)nb);
  or_srand(seed);
  or_shuffle_pairs(nb, o1, o2);
  tbonds = (int)(pb * (double)nb);
  if (literal)
    cln = or_label_bonds_literal(lattice, m, n, pbc, nb, b1, b2, o1, o2, tbonds,
                                 label, csize, &res->maxcn, &res->maxcs);
  else
    cln = or_label_bonds_replay(lattice, m, n, pbc, nb, b1, b2, o1, o2, tbonds,
                                label, csize, &res->maxcn, &res->maxcs);
  res->nb = nb;
  res->tbonds = tbonds;
  res->cln = cln;
  if (cln < 0) return cln;
  res->perccln = or_span_bonds(m, n, nb, b1, b2, label, csize, cln);
  res->perccls = res->perccln ? csize[res->perccln] : 0;
  if (res->perccln > 0) {
    double *gval = (double *)malloc(sizeof(double) * (size_t)nb);
    double *diag = (double *)malloc(sizeof(double) * (size_t)t);
    double *itemp = (double *)malloc(sizeof(double) * (size_t)N);
    double *vint = (double *)calloc((size_t)N, sizeof(double));
    int nmax = N + 1 + 2 * nb + 8;
    double *sa = (double *)calloc((size_t)nmax, sizeof(double));
    int *ija = (int *)calloc((size_t)nmax, sizeof(int));
    or_bond_values(0, nb, b1, b2, label, NULL, res->perccln, g0, 1.0e-12, gval);
    or_assemble(lattice, m, n, pbc, nb, b1, b2, gval, Va, 1.0e-16, 0, nmax, sa,
                ija, itemp, diag);
    or_linbcg(sa, ija, N, itemp, vint, 2, tol, itmax, &res->iter, &res->err,
              NULL);
    or_currents(lattice, m, n, pbc, nb, b1, b2, gval, diag, vint, Va, 1.0e-10,
                0, &res->gtop, &res->gbot);
    free(gval); free(diag); free(itemp); free(vint); free(sa); free(ija);
  }
  if (o1_out) memcpy(o1_out, o1, sizeof(int) * (size_t)(nb + 1));
  if (o2_out) memcpy(o2_out, o2, sizeof(int) * (size_t)(nb + 1));
  free(b1); free(b2); free(o1); free(o2);
  if (!label_out) free(label);
  if (!csize_out) free(csize);
  return 0;
}

/* ======================================================================
 * One bond_cond trial (Square/bond_cond.f:123-498): every bond of the
 * shuffled order is added with the literal loop, the spanning scan runs
 * after each addition (:353-389) and the conductance is computed when
 * bf == nbarr(jj) (:392-483).  pb grid: pbarr(1)=0.49, +5e-3 to index 103,
 * nbarr = int(pbarr*nb) (:84-97; repeated values stall the sweep, H3);
 * triangular: pbarr(1)=0.35, 131 points.
 * ==================================================================== */
int or_bond_cond_trial(int lattice, int m, int n, int pbc, int tseed,
                       double Va, double g0, int itmax, double tol,
                       double *row_pb, double *row_gbot, double *row_gtop,
                       int *row_iter, int *perccln_out, double *pc_out) {
  int t = m * n, nb = or_nbonds(lattice, m, n, pbc), N = t - 2 * m;
  int *b1 = (int *)malloc(sizeof(int) * (size_t)nb);
  int *b2 = (int *)malloc(sizeof(int) * (size_t)nb);
  int *o1 = (int *)calloc((size_t)nb + 1, sizeof(int));
  int *o2 = (int *)calloc((size_t)nb + 1, sizeof(int));
  int *label = (int *)calloc((size_t)nb, sizeof(int));
  int *csize = (int *)calloc((size_t)nb + 2, sizeof(int));
  double pbarr[250];
  int nbarr[250], i, jj = 0, bf = 0, perccln = 0, nrows = 0;
  double pc = 0.0;
  lit_state S;
  if (or_bond_list(lattice, m, n, pbc, b1, b2) != nb) return -1;
  for (i = 0; i < 250; i++) { pbarr[i] = 0.0; nbarr[i] = 0; }
  /* Square/bond_cond.f:91-94 (0.49, 103 points);
     Triangular/bond_cond.f:91-94 (0.35, 131 points) */
  pbarr[0] = lattice ? 0.35 : 0.49;
  for (i = 1; i < (lattice ? 131 : 103); i++) pbarr[i] = pbarr[i - 1] + 5.00e-03;
  for (i = 0; i < 250; i++) nbarr[i] = (int)(pbarr[i] * (double)nb);
  memcpy(o1, b1, sizeof(int) * (size_t)nb);
  memcpy(o2, b2, sizeof(int) * (size_t)nb);
  or_srand(tseed);
  or_shuffle_pairs(nb, o1, o2);
  S.lattice = lattice; S.m = m; S.n = n; S.pbc = pbc; S.nb = nb;
  S.scn = or_scn(lattice); S.bcn = or_bcn(lattice);
  S.b1 = b1; S.b2 = b2; S.label = label; S.csize = csize;
  S.cln = 1; S.maxcn = 0; S.maxcs = 0;
  for (i = 1; i <= nb; i++) {
    int sp;
    float pbf;
    lit_add_bond(&S, o1[i - 1], o2[i - 1]);
    bf = bf + 1;
    pbf = (float)bf / (float)nb;
    sp = or_span_bonds(m, n, nb, b1, b2, label, csize, S.cln);
    if (sp > 0) {
      if (perccln == 0) pc = (double)pbf;
      perccln = sp;
    }
    if (jj < 250 && bf == nbarr[jj]) {
      double gtop = 0.0, gbot = 0.0;
      int iter = 0;
      if (perccln > 0) {
        double *gval = (double *)malloc(sizeof(double) * (size_t)nb);
        double *diag = (double *)malloc(sizeof(double) * (size_t)t);
        double *itemp = (double *)malloc(sizeof(double) * (size_t)N);
        double *vint = (double *)calloc((size_t)N, sizeof(double));
        int nmax = N + 1 + 2 * nb + 8;
        double *sa = (double *)calloc((size_t)nmax, sizeof(double));
        int *ija = (int *)calloc((size_t)nmax, sizeof(int));
        double err;
        or_bond_values(0, nb, b1, b2, label, NULL, perccln, g0, 1.0e-12, gval);
        or_assemble(lattice, m, n, pbc, nb, b1, b2, gval, Va, 1.0e-16, 0, nmax,
                    sa, ija, itemp, diag);
        or_linbcg(sa, ija, N, itemp, vint, 2, tol, itmax, &iter, &err, NULL);
        or_currents(lattice, m, n, pbc, nb, b1, b2, gval, diag, vint, Va,
                    1.0e-10, 0, &gtop, &gbot);
        free(gval); free(diag); free(itemp); free(vint); free(sa); free(ija);
      }
      jj++;
      row_pb[nrows] = (double)pbf;
      row_gbot[nrows] = gbot;
      row_gtop[nrows] = gtop;
      if (row_iter) row_iter[nrows] = iter;
      nrows++;
    }
  }
  *perccln_out = perccln;
  *pc_out = pc;
  free(b1); free(b2); free(o1); free(o2); free(label); free(csize);
  return nrows;
}
