// perc_assemble.hip -- Kirchhoff assembly and terminal currents of libperc
// (gfx950): the interior system of the spanning cluster as stencil row codes
// and / or CSR (Square/bondc.f:482-538, ConductCalc.m:88-165), bond weights,
// and the currents into the electrodes (bondc.f:554-592).  Every
// floating-point operation in the reference's order (-ffp-contract=off).
#include "perc_stencil.h"

namespace perc {
namespace {

// ---------------------------------------------------------------------------
// Kirchhoff assembly (bondc.f:482-538, ConductCalc.m:88-165)
// w (optional): ConductCalc.m condtype 2, G = -g0*rand for the bonds of the
// spanning cluster (ConductCalc.m:94-97): per-bond multipliers w[id]
__device__ __forceinline__ double bond_value(int rule, int id, int s, int c, int ps,
                                             const uint8_t* bocc, const uint8_t* socc,
                                             int span_root, double g0, double leak,
                                             const double* w) {
  bool in;
  if (rule == PERC_RULE_BOND) in = bocc[id] && ps == span_root;
  else if (rule == PERC_RULE_SITE) in = socc[s] && socc[c] && ps == span_root;
  else in = bocc[id] && socc[s] && socc[c] && ps == span_root;
  return in ? (w ? -g0 * w[id] : -g0) : -leak;
}

// CSR: also the NR-ordered CSR values and the diagonal array (the CSR and
// split formats, perc_get_system, the probes).  The stencil solvers read
// only code and rhs, so dev_assemble writes the CSR copy only when a
// consumer asks for it (ensure_csr): 2 + 8 B per row instead of 50.
template <bool CSR>
__device__ __forceinline__ void assemble_row(
    const Geom& g, int i, const int* bond_first, const uint8_t* bocc, const uint8_t* socc,
    const int* parent, const int* rowptr, double* val, double* diag, double* rhs, uint16_t* code,
    int* sflag, const StencilForms& F, int fast_form, int fast_l, int fast_r, int bf_closed,
    int rule, double g0,
    double leak, double Va, int span_root, const double* w) {
  const int m = g.m, t = g.t, s = i + m + 1;
  const int ps = parent[s];
  const int sr = div_m(g, s - 1), sc = s - 1 - sr * m;
  // Square lattice, closed forms (the host found each form in the table and
  // checked its deltas): the sorted neighbours and their bond ids follow
  // from nearestn_square case by case --
  //   interior column: s-m, s-1, s+1, s+m; ids bf(s-m)+1, bf(s-1), fb, fb+1
  //     (s is the 2nd forward neighbour of s-m, the 1st of s-1 -- every
  //     nearestn_square case lists +1 before +m);
  //   column 0: s-m, s+1, [s+m-1 (pbc)], s+m; ids bf(s-m)+1, fb, [fb+2], fb+1
  //     (s's forward order is s+1, s+m, s+m-1);
  //   column m-1: s-m, [s-m+1 (pbc)], s-1, s+m; ids bf(s-m), [bf(s-m+1)+2],
  //     bf(s-1), fb (s-m's only forward neighbour is s; s is the 3rd of s-m+1).
  // RHS (top system row): the one forward neighbour above, s+m (the pbc
  // wrap neighbour s+m-1 of column 0 is in s's own row).  Every load is issued before any
  // is used (bond_value's short-circuit loads would serialise the latencies).
  const int kind_c = sc >= 1 && sc <= m - 2 ? 0 : (sc == 0 ? 1 : 2);
  const int cform = kind_c == 0 ? fast_form : kind_c == 1 ? fast_l : fast_r;
  if (cform >= 0) {
    const bool pb = g.pbc != 0;
    int fb, bl, bd, bw = 0;  // bond_first of s, s-1, s-m, s-m+1
    if (bf_closed) {
      fb = bf_square(g, sr, sc);
      bl = sc > 0 ? bf_square(g, sr, sc - 1) : 0;
      bd = bf_square(g, sr - 1, sc);
      bw = bf_square(g, sr, 0);
    } else {
      fb = bond_first[s];
      bl = sc > 0 ? bond_first[s - 1] : 0;
      bd = bond_first[s - m];
      bw = kind_c == 2 && pb ? bond_first[s - m + 1] : 0;
    }
    int cs[4], ids[4], cnt;
    if (kind_c == 0) {
      cnt = 4;
      cs[0] = s - m; cs[1] = s - 1; cs[2] = s + 1; cs[3] = s + m;
      ids[0] = bd + 1; ids[1] = bl; ids[2] = fb; ids[3] = fb + 1;
    } else if (kind_c == 1) {
      cnt = pb ? 4 : 3;
      cs[0] = s - m; cs[1] = s + 1; cs[2] = pb ? s + m - 1 : s + m; cs[3] = s + m;
      ids[0] = bd + 1; ids[1] = fb; ids[2] = pb ? fb + 2 : fb + 1; ids[3] = fb + 1;
    } else {
      cnt = pb ? 4 : 3;
      cs[0] = s - m; cs[1] = pb ? s - m + 1 : s - 1; cs[2] = pb ? s - 1 : s + m; cs[3] = s + m;
      ids[0] = bd; ids[1] = pb ? bw + 2 : bl; ids[2] = pb ? bl : fb; ids[3] = fb;
    }
    unsigned bo[4], so[4] = {1u, 1u, 1u, 1u}, ss = 1u;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bo[j] = rule == PERC_RULE_SITE ? 1u : bocc[ids[j]];
    if (rule != PERC_RULE_BOND) {
      ss = socc[s];
#pragma unroll
      for (int j = 0; j < 4; ++j) so[j] = socc[cs[j]];
    }
    const bool root = ps == span_root;
    double gvs[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // bond_value
      const bool in = root && bo[j] != 0u && ss != 0u && so[j] != 0u;
      gvs[j] = in ? (w ? -g0 * w[ids[j]] : -g0) : -leak;
    }
    double rowsum = 0.0;
    unsigned bits = 0;
    int k = CSR ? rowptr[i] : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= cnt) break;
      const double gv = gvs[j];
      if (gv == -g0) bits |= 1u << j;
      rowsum = rowsum + gv;
      if (CSR && cs[j] > m && cs[j] <= t - m) val[k++] = gv;
    }
    code[i] = (uint16_t)(bits | (unsigned)cnt << 8 | (unsigned)cform << 11);
    if (CSR) diag[i] = -rowsum;
    double acc = 0.0;
    if (s > t - 2 * m) acc = acc - (gvs[cnt - 1] * Va);  // (s, s+m): the last slot
    rhs[i] = acc;
    return;
  }
  // one division per neighbour (div_m); nearestn of the row once and of
  // each smaller neighbour once -- the bond ids of bond_id
  int nn[6];
  nearestn_rc(g, s, sr, sc, nn);
  const int fb = bond_first[s];
  int nbr[6], cnt = 0;  // sorted_neighbours
  for (int k = 0; k < g.scn; ++k)
    if (nn[k] != 0) {
      const int v = nn[k];
      int j = cnt;
      while (j > 0 && nbr[j - 1] > v) { nbr[j] = nbr[j - 1]; --j; }
      nbr[j] = v;
      ++cnt;
    }
  double rowsum = 0.0;  // bondc.f:500-504: ascending-column dense row sum
  int k = CSR ? rowptr[i] : 0;
  unsigned bits = 0;
  int drs[6], dcs[6];
  for (int j = 0; j < cnt; ++j) {
    const int c = nbr[j];
    const int cr = div_m(g, c - 1), cc = c - 1 - cr * m;
    int d = cc - sc;  // lattice_delta
    if (d > 1) d -= m;
    else if (d < -1) d += m;
    drs[j] = cr - sr;
    dcs[j] = d;
    int id;
    if (s < c) {
      id = fwd_bond_id(g, nn, fb, s, c);
    } else {
      int nc[6];
      nearestn_rc(g, c, cr, cc, nc);
      id = fwd_bond_id(g, nc, bond_first[c], c, s);
    }
    if (id < 0) {  // no bond in this slot: the stencil operator cannot be used
      atomicOr(sflag, 1);
      continue;
    }
    const double gv = bond_value(rule, id, s, c, ps, bocc, socc, span_root, g0, leak, w);
    if (gv == -g0) bits |= 1u << j;
    rowsum = rowsum + gv;
    if (CSR && c > m && c <= t - m) val[k++] = gv;
  }
  int form = -1;  // the row's form: same count and offsets
  for (int f = 0; f < F.nforms && form < 0; ++f) {
    bool same = F.cnt[f] == cnt;
    for (int j = 0; j < cnt && same; ++j) same = F.off[f][j] == nbr[j] - s;
    if (same) form = f;
  }
  if (form < 0) {
    atomicOr(sflag, 2);
    form = 0;
  }
  for (int j = 0; j < cnt; ++j) {  // the tiled kernel reads slot j at (row, col) + (dr, dc)
    const int dr = drs[j], dc = dcs[j];
    if (dr != F.dr[form][j] || dc != F.dc[form][j] || dr < -1 || dr > 1 || dc < -1 || dc > 1)
      atomicOr(sflag, 4);
  }
  code[i] = (uint16_t)(bits | (unsigned)cnt << 8 | (unsigned)form << 11);
  if (CSR) diag[i] = -rowsum;
  // RHS in bond-list order (bondc.f:490-497)
  double acc = 0.0;
  if (s > t - 2 * m && s <= t - m) {
    int r = 0;
    for (int kk = 0; kk < g.scn; ++kk) {
      const int q = nn[kk];
      if (q <= s) continue;
      if (q > t - m) {
        const double gv =
            bond_value(rule, fb + r, s, q, ps, bocc, socc, span_root, g0, leak, w);
        acc = acc - (gv * Va);
      }
      ++r;
    }
  }
  rhs[i] = acc;
}

// One row per thread (a grid-stride loop measured 1.65x slower: each
// iteration's loads wait for the last's, fewer rows in flight).  The
// StencilForms table (~900 B) is read through a device pointer by the
// general path only: as a kernel argument every wave would s_load it.
template <bool CSR>
__global__ __launch_bounds__(kBlock) void k_assemble(
    Geom g, int N, const int* bond_first, const uint8_t* bocc, const uint8_t* socc,
    const int* parent, const int* rowptr, double* val, double* diag, double* rhs, uint16_t* code,
    int* sflag, const StencilForms* F, int fast_form, int fast_l, int fast_r, int bf_closed,
    int rule, double g0,
    double leak, double Va, int span_root, const double* w) {
  // XCD-contiguous row blocks: in dispatch order the lattice's edge-column
  // workgroups (general path, ~6x the closed form's work) are every 16th at
  // m = 4096 -- all on one XCD, the kernel waited on it (+120 us at L = 4096)
  const int i = xcd_logical_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (i == 0 && w) atomicOr(sflag, 1);  // per-bond values: no two-value stencil code
  // a workgroup with a general-path row (an edge column, a triangular or
  // non-closed-form lattice) stages the form table in LDS first: read from
  // global memory inside the general path's loops it was a chain of
  // dependent loads, ~100 us of latency per such wave -- the kernel's tail
  __shared__ StencilForms sF;
  bool gen = false;
  if (i < N) {
    const int s = i + g.m + 1, sr = div_m(g, s - 1), sc = s - 1 - sr * g.m;
    const int f = sc >= 1 && sc <= g.m - 2 ? fast_form : (sc == 0 ? fast_l : fast_r);
    gen = f < 0;
  }
  if (__syncthreads_or(gen)) {
    static_assert(sizeof(StencilForms) % 4 == 0, "word copy");
    const int nw = (int)(sizeof(StencilForms) / 4);
    const int* src = reinterpret_cast<const int*>(F);
    int* dst = reinterpret_cast<int*>(&sF);
    for (int k = threadIdx.x; k < nw; k += blockDim.x) dst[k] = src[k];
    __syncthreads();
  }
  if (i >= N) return;
  assemble_row<CSR>(g, i, bond_first, bocc, socc, parent, rowptr, val, diag, rhs, code, sflag, sF,
                    fast_form, fast_l, fast_r, bf_closed, rule, g0, leak, Va, span_root, w);
}

// Terminal currents of the 2m boundary rows (bondc.f:554-592; ConductCalc.m:188)
__global__ void k_currents(Geom g, const int* bond_first, const uint8_t* bocc,
                           const uint8_t* socc, const int* parent, const double* x, int rule,
                           int cur_rule, double g0, double leak, double Va, int span_root,
                           double thresh, double* iout, const double* w) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int m = g.m, t = g.t;
  if (idx >= 2 * m) return;
  const int s = idx < m ? idx + 1 : t - m + 1 + (idx - m);
  const int ps = parent[s];
  int nbr[6];
  const int cnt = sorted_neighbours(g, s, nbr);
  double gv[6];
  double rowsum = 0.0;
  for (int j = 0; j < cnt; ++j) {
    const int c = nbr[j];
    const int id = s < c ? bond_id(g, bond_first, s, c) : bond_id(g, bond_first, c, s);
    gv[j] = id < 0 ? 0.0 : bond_value(rule, id, s, c, ps, bocc, socc, span_root, g0, leak, w);
    rowsum = rowsum + gv[j];
  }
  const double d = -rowsum;
  auto V = [&](int c) -> double { return c <= m ? 0.0 : (c > t - m ? Va : x[c - m - 1]); };
  double acc;
  if (cur_rule == PERC_CUR_FORTRAN) {
    acc = d * V(s);
    for (int j = 0; j < cnt; ++j)
      if (fabs(gv[j]) >= thresh) acc = acc + gv[j] * V(nbr[j]);
  } else {
    acc = 0.0;
    bool done = false;
    for (int j = 0; j < cnt; ++j) {
      if (!done && nbr[j] > s) { acc = acc + d * V(s); done = true; }
      acc = acc + gv[j] * V(nbr[j]);
    }
    if (!done) acc = acc + d * V(s);
  }
  iout[idx] = acc;
}

}  // namespace

// Row forms of the interior system (sorted neighbour offsets c - s).  A
// row's form depends only on its column and the parity of its lattice row,
// so the first two interior rows hold every form; the assembly checks each
// row against the table anyway (sflag bit 2).
StencilForms stencil_forms(const Geom& g) {
  StencilForms F{};
  const int rows = std::min(2, g.n - 2);
  for (int r = 1; r <= rows; ++r)
    for (int cx = 0; cx < g.m; ++cx) {
      const int s = r * g.m + cx + 1;
      int nb[6];
      const int cnt = sorted_neighbours(g, s, nb);
      int f = 0;
      for (; f < F.nforms; ++f) {
        bool same = F.cnt[f] == cnt;
        for (int j = 0; j < cnt && same; ++j) same = F.off[f][j] == nb[j] - s;
        if (same) break;
      }
      if (f < F.nforms) continue;
      if (F.nforms == kMaxForms) return StencilForms{};  // no stencil operator
      F.cnt[f] = cnt;
      for (int j = 0; j < kMaxSlots; ++j) {
        F.off[f][j] = j < cnt ? nb[j] - s : 0;
        F.dr[f][j] = F.dc[f][j] = 0;
        if (j < cnt) lattice_delta(g, s, nb[j], &F.dr[f][j], &F.dc[f][j]);
      }
      ++F.nforms;
    }
  for (int f = 0; f < F.nforms; ++f) {
    F.regular[f] = 1;
    int last = -1;
    for (int j = 0; j < F.cnt[f]; ++j) {
      const int dr = F.dr[f][j], dc = F.dc[f][j];
      if (dr < -1 || dr > 1 || dc < -1 || dc > 1 || (dr == 0 && dc == 0)) {
        F.regular[f] = 0;  // not a 3x3 stencil: the tiled kernels are not used
        continue;
      }
      const int k9 = (dr + 1) * 3 + (dc + 1), kp = k9 < 4 ? k9 : k9 - 1;
      F.rpos[f] |= (unsigned)kp << (3 * j);
      F.rmask[f] |= 1u << kp;
      if (kp <= last) F.regular[f] = 0;
      last = kp;
    }
    F.rmap[f] = kRmapIrregular;
    if (F.regular[f]) {
      F.rmap[f] = 0xFFFFFFFFu;
      for (int j = 0; j < F.cnt[f]; ++j) {
        const unsigned kp = (F.rpos[f] >> (3 * j)) & 7u;
        F.rmap[f] &= ~(0xFu << (4 * kp));
        F.rmap[f] |= (unsigned)j << (4 * kp);
      }
      F.umask |= F.rmask[f];
    }
  }
  return F;
}

static // The CSR rows of <= 4 off-diagonals in 4 aligned slots, in the CSR order:
// columns (padding: the row itself), values (padding: 0, never added), the
// entry count (perc_csr.h ell_row)
__global__ __launch_bounds__(kBlock) void k_csr_to_ell(int N, const int* __restrict__ rowptr,
                                                       const int* __restrict__ col,
                                                       const double* __restrict__ val, int4* ecol,
                                                       double2* eval, uint8_t* ecnt) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= N) return;
  const int a = rowptr[i], n = rowptr[i + 1] - a;
  int c[4];
  double v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = j < n ? col[a + j] : i;
    v[j] = j < n ? val[a + j] : 0.0;
  }
  ecol[i] = make_int4(c[0], c[1], c[2], c[3]);
  eval[2 * i] = make_double2(v[0], v[1]);
  eval[2 * i + 1] = make_double2(v[2], v[3]);
  ecnt[i] = (uint8_t)n;
}

hipError_t launch_assemble(perc_ctx* h, bool csr) {
  HIP_TRY(dev_flatten(h));  // (the roots, not their ancestors)
  DeviceBuffers& d = h->d;
  const AsmParams& p = h->asm_p;
  hipStream_t st = h->stream;
  HIP_TRY(hipMemsetAsync(d.sflag, 0, 4 * sizeof(int), st));
  const double* w = h->has_weights ? d.bw : nullptr;
  // the square lattice's interior-column form (k_assemble's closed-form path)
  int fast = -1;
  const StencilForms& F = h->forms;
  const int m = h->g.m;
  const char* gen = std::getenv("PERC_ASM_GENERIC");  // tests: the general path only
  const bool closed = !(gen && gen[0] == '1');
  // the closed-form rows' forms (k_assemble): offsets and lattice deltas of
  // the interior, column-0 and column-(m-1) rows of the square lattice
  auto find_form = [&](int cnt, const int* off, const int* dr, const int* dc) {
    for (int f = 0; f < F.nforms; ++f) {
      bool same = F.cnt[f] == cnt;
      for (int j = 0; j < cnt && same; ++j)
        same = F.off[f][j] == off[j] && F.dr[f][j] == dr[j] && F.dc[f][j] == dc[j];
      if (same) return f;
    }
    return -1;
  };
  int fl = -1, fr = -1;
  h->nib_ok = false;
  if (closed && h->g.lattice == kSquare && m >= 4) {
    const int oi[4] = {-m, -1, 1, m}, ri[4] = {-1, 0, 0, 1}, ci[4] = {0, -1, 1, 0};
    fast = find_form(4, oi, ri, ci);
    if (h->g.pbc) {
      const int ol[4] = {-m, 1, m - 1, m}, rl[4] = {-1, 0, 0, 1}, cl[4] = {0, 1, -1, 0};
      const int orr[4] = {-m, -(m - 1), -1, m}, rr[4] = {-1, 0, 0, 1}, cr[4] = {0, 1, -1, 0};
      fl = find_form(4, ol, rl, cl);
      fr = find_form(4, orr, rr, cr);
    } else {
      const int ol[3] = {-m, 1, m}, rl[3] = {-1, 0, 1}, cl[3] = {0, 1, 0};
      const int orr[3] = {-m, -1, m}, rr[3] = {-1, 0, 1}, cr[3] = {0, -1, 0};
      fl = find_form(3, ol, rl, cl);
      fr = find_form(3, orr, rr, cr);
    }
    // the column classes of the nibble codes (k_pack_nib checks every row)
    const unsigned ce = h->g.pbc ? 4u : 3u;
    h->ncls[0] = 4u << 8 | (unsigned)fast << 11;
    h->ncls[1] = ce << 8 | (unsigned)fl << 11;
    h->ncls[2] = ce << 8 | (unsigned)fr << 11;
    h->nib_ok = fast >= 0 && fl >= 0 && fr >= 0 && m % 2 == 0;
  }
  if (csr)
    k_assemble<true><<<cdiv(h->N, kBlock), kBlock, 0, st>>>(h->g, h->N, d.bond_first, d.bocc, d.socc,
                                                          d.parent, d.rowptr, d.val, d.diag, d.rhs,
                                                          d.code, d.sflag, d.forms_dev, fast, fl, fr, (int)h->bf_closed, p.rule,
                                                          p.g0, p.leak, p.Va, p.span_root, w);
  else
    k_assemble<false><<<cdiv(h->N, kBlock), kBlock, 0, st>>>(h->g, h->N, d.bond_first, d.bocc, d.socc,
                                                           d.parent, d.rowptr, d.val, d.diag, d.rhs,
                                                           d.code, d.sflag, d.forms_dev, fast, fl, fr, (int)h->bf_closed, p.rule,
                                                           p.g0, p.leak, p.Va, p.span_root, w);
  HIP_TRY(dbg_sync(st, "k_assemble"));
  h->csr_ok = csr;
  h->ell_ok = false;
  if (csr && h->csr_maxrow <= 4) {  // the ELL copy the CSR SpMV kernels read (perc_csr.h ell_row)
    if (!d.ell_col) {
      HIP_TRY(hipMalloc(&d.ell_col, sizeof(int4) * (size_t)h->N));
      HIP_TRY(hipMalloc(&d.ell_val, sizeof(double2) * 2 * (size_t)h->N));
      HIP_TRY(hipMalloc(&d.ell_cnt, (size_t)h->N));
    }
    k_csr_to_ell<<<cdiv(h->N, kBlock), kBlock, 0, st>>>(h->N, d.rowptr, d.col, d.val, d.ell_col, d.ell_val,
                                                       d.ell_cnt);
    HIP_TRY(dbg_sync(st, "k_csr_to_ell"));
    h->ell_ok = true;
  }
  return hipSuccess;
}

// the CSR copy of the assembled system (values, diagonal), for the
// consumers that read it; the stencil assembly leaves it unwritten
hipError_t ensure_csr(perc_ctx* h) {
  if (h->csr_ok || !h->assembled || !h->asm_p.valid) return hipSuccess;
  return launch_assemble(h, true);
}

hipError_t dev_assemble(perc_ctx* h, int rule, double g0, double leak, double Va, int span_root) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  h->asm_p = AsmParams{true, rule, span_root, g0, leak, Va};
  // per-bond weights take the CSR operator (two-value stencil codes cannot
  // hold them): assemble the CSR copy at once; else the stencil rows only,
  // and the CSR copy after all if a row does not fit a stencil form
  HIP_TRY(launch_assemble(h, h->has_weights));
  int flag = 0;
  HIP_TRY(hipMemcpyAsync(&flag, d.sflag, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  h->st_ng0 = -g0;
  h->st_nleak = -leak;
  if (d.dtab) {
    k_fill_dtab<<<cdiv(kDiagTab, kBlock), kBlock, 0, st>>>(d.dtab, -g0, -leak);
    HIP_TRY(hipGetLastError());
  }
  h->stencil_ok = (flag & 3) == 0 && h->forms.nforms > 0;
  h->tiled_ok = h->stencil_ok && (flag & 4) == 0 && h->tile_grid > 0 && h->g.m % 2 == 0;
  h->march_ok = h->tiled_ok && h->march_grid > 0;
  select_format(h);
  if (!h->stencil_ok) HIP_TRY(launch_assemble(h, true));
  return hipSuccess;
}

hipError_t dev_currents(perc_ctx* h, int rule, int cur_rule, double g0, double leak, double Va,
                        int span_root, double thresh, double* iout_host) {
  HIP_TRY(dev_flatten(h));
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  const int m = h->g.m;
  k_currents<<<blocks_for(2 * m), kBlock, 0, st>>>(h->g, d.bond_first, d.bocc, d.socc, d.parent,
                                                    d.x, rule, cur_rule, g0, leak, Va, span_root,
                                                    thresh, d.iout, h->has_weights ? d.bw : nullptr);
  HIP_TRY(dbg_sync(st, "k_currents"));
  HIP_TRY(hipMemcpyAsync(iout_host, d.iout, sizeof(double) * 2 * m, hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

// the bonds the assembly gives -g0 (bond_value's "in"), one byte per bond in
// bond-list order: ConductCalc.m condtype 2 draws one rand per such bond
// (perc_set_conductcalc_weights)
__global__ void k_bond_mask(Geom g, int rule, const int* bond_first, const uint8_t* bocc,
                            const uint8_t* socc, const int* parent, int span_root, uint8_t* mask) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (s > g.t - 1) return;
  const int row = div_m(g, s - 1);
  int nn[6];
  nearestn_rc(g, s, row, s - 1 - row * g.m, nn);
  const int fb = bond_first[s];
  int r = 0;
  for (int k = 0; k < g.scn; ++k) {
    const int q = nn[k];
    if (q <= s) continue;
    const int id = fb + r++;
    bool in;
    if (rule == PERC_RULE_BOND) in = bocc[id] && parent[s] == span_root;
    else if (rule == PERC_RULE_SITE) in = socc[s] && socc[q] && parent[s] == span_root;
    else in = bocc[id] && socc[s] && socc[q] && parent[s] == span_root;
    mask[id] = in ? 1 : 0;
  }
}

hipError_t dev_bond_mask(perc_ctx* h, int rule, uint8_t* mask_host) {
  HIP_TRY(dev_flatten(h));  // (the roots, not their ancestors)
  DeviceBuffers& d = h->d;
  uint8_t* dm = nullptr;
  HIP_TRY(dmalloc(&dm, (size_t)h->nb + 8));
  k_bond_mask<<<blocks_for(h->g.t), kBlock, 0, h->stream>>>(h->g, rule, d.bond_first, d.bocc, d.socc, d.parent,
                                                           h->span_root, dm);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(mask_host, dm, (size_t)h->nb, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(dm);
  return e;
}

hipError_t dev_set_bond_weights(perc_ctx* h, const double* w) {
  DeviceBuffers& d = h->d;
  // the assembled system (its stencil codes, rhs, the CSR copy ensure_csr
  // would re-assemble from the current weights) no longer matches: assemble
  // again before the next solve / system read
  h->assembled = false;
  h->csr_ok = false;
  h->ell_ok = false;
  if (!w) {
    h->has_weights = false;
    return hipSuccess;
  }
  if (!d.bw) HIP_TRY(dmalloc(&d.bw, (size_t)h->nb + 8));
  HIP_TRY(hipMemcpy(d.bw, w, sizeof(double) * h->nb, hipMemcpyHostToDevice));
  h->has_weights = true;
  return hipSuccess;
}

}  // namespace perc
